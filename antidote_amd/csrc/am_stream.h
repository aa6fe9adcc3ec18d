// am_stream.h -- the streaming materialize kernel of the PN counter and the LWW register.
//
// Work split.  Reads are cut into batches of 64 consecutive reads; wavefront gw
// of W takes batches gw, gw+W, gw+2W, ...  For a batch, lane i loads read i's
// metadata with one vector load (key, key_off[key], key_off[key+1], key_type),
// so no dependent global load sits on the per-read critical path, and lane i
// also BUFFERS read i's outputs: after a read is reduced, its wave-uniform
// results are parked in lane i's registers, and the batch's results leave with
// one coalesced vector store per output column (64 consecutive reads).  Scattered
// single-lane stores of each result cost 20% of the kernel (measured, r01).
//
// Streaming.  The wave walks its reads' op logs as one stream of 256-op tiles
// (lane l owns 4 consecutive ops of a tile: 16-byte loads, one contiguous 1-2 KiB
// segment per column per wave instruction) and double-buffers it: the next tile's
// loads (possibly the next read's, or the next batch's, first tile) are issued
// before the current tile is evaluated and its read reduced (DPP row butterflies +
// 4 readlanes).  The next batch's metadata is prefetched one batch ahead, so the
// stream does not drain at batch boundaries.
//
// Packed view (am_pack.hip): the tile streams the op's commit vector as u32 entries relative
// to the key's time base (4*D + payload bytes per op instead of 9 + 8*D + payload) and the
// inclusion test runs on u32 (am_wave.h pk_eval); escaped ops are read from the full columns.
//
// Per-op semantics: am_wave.h eval_op (is_op_in_snapshot/7, belongs_to_snapshot_op/3).
// Per-read outputs: materialize/4's {ok, Value, NewLastOp, LastOpCt, IsNewSS, Count}.
#pragma once
#include "am_wave.h"

namespace amk_stream {
using namespace amk;

constexpr int BLOCK = 256;
constexpr int WPB = BLOCK / WAVE;
// ops per lane of a tile: 4 (16-byte loads), 2 for 8-DC clocks (measured: C3 11.8 -> 11.2 ms;
// at D = 16 the narrower tile was slower, 4.2 -> 4.7 ms), which shrinks the double-buffered tiles
template <int DMAX>
constexpr int opl_of() { return DMAX == 8 ? 2 : 4; }

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
template <int N>
__device__ __forceinline__ void ld_u64(const uint64_t *p, uint64_t *o) {
  const u64x2 a = *(const u64x2 *)p;
  o[0] = a.x, o[1] = a.y;
  if constexpr (N == 4) {
    const u64x2 b = *(const u64x2 *)(p + 2);
    o[2] = b.x, o[3] = b.y;
  }
}
template <int N>
__device__ __forceinline__ void ld_u32(const uint32_t *p, uint32_t *o) {
  if constexpr (N == 4) {
    const u32x4 a = *(const u32x4 *)p;
    o[0] = a.x, o[1] = a.y, o[2] = a.z, o[3] = a.w;
  } else {
    const u32x2 a = *(const u32x2 *)p;
    o[0] = a.x, o[1] = a.y;
  }
}

template <int DMAX, int OPL = opl_of<DMAX>()>
struct Tile {
  uint32_t meta4;           // full view
  uint64_t ct[OPL];
  uint64_t sv[OPL][DMAX];
  uint32_t x[OPL][DMAX];    // packed view (am_pack.hip): X[d] - key_tbase
  uint32_t sp[OPL];
  uint64_t p0[OPL], p1[OPL], tx[OPL];
};

// per-lane buffered outputs of read (batch base + lane)
template <int DMAX>
struct Out {
  int32_t status;
  uint32_t flags, pres, count;
  uint32_t ign, newss, vflag;
  int64_t nlo;
  uint64_t ct[DMAX];  // only with BUF_CT
  uint64_t v0, v1;
  uint32_t fin;       // the read was finalized (wide clocks: LastOpCt already stored)
};

template <int TYPE>
struct SOf {
  using T = typename ValOf<TYPE>::T;
  static constexpr bool NEED_P0 = true, NEED_P1 = ValOf<TYPE>::NEED_P1;
};

template <int DMAX, int TYPE, bool GENERAL, bool PACKED>
__global__ void __launch_bounds__(BLOCK) k_stream(am_op_log L, am_read_batch B, am_read_result R, am_sel S,
                                                  am_rows_cfg H) {
  using V = typename SOf<TYPE>::T;
  constexpr int OPL = opl_of<DMAX>();
  constexpr uint64_t TILE = (uint64_t)WAVE * OPL;
  constexpr bool BUF_CT = DMAX < 8;  // wide clocks: LastOpCt leaves at finalize (fewer VGPRs)
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  const uint64_t n = B.n_reads;  // column stride of per-read arrays
  // reads to process: slots [0, nsel) -> read sbase[slot] (or the identity)
  const uint32_t sel0 = S.idx ? uniform_u32(S.range[0]) : 0u;
  const uint64_t nsel = S.idx ? (uint64_t)(uniform_u32(S.range[1]) - sel0) : n;
  const uint32_t *sbase = S.idx ? S.idx + sel0 : nullptr;
  const uint32_t nd = L.n_dc;
  const uint64_t stride = L.snap_stride ? L.snap_stride : L.n_ops;
  const uint64_t W = (uint64_t)gridDim.x * WPB;
  const uint64_t gw = (uint64_t)blockIdx.x * WPB + uniform_u32(threadIdx.x >> 6);
  const uint64_t n_batches = (nsel + WAVE - 1) / WAVE;
  if (gw >= n_batches) return;

  ReadU<DMAX> u;
  u.allmask = nd >= 32 ? 0xFFFFFFFFu : ((1u << nd) - 1u);
  u.base_ignore = true;
  u.has_txid = false;
  u.txid = 0;
  u.cpres = 0;
#pragma unroll
  for (int d = 0; d < DMAX; ++d) u.C0[d] = 0;
  auto load_clock = [&](uint64_t ridx, uint64_t rstride) {
    u.spres = uniform_u32(B.read_pres[ridx]) & u.allmask;
#pragma unroll
    for (int d = 0; d < DMAX; ++d)
      u.S[d] = (d < (int)nd && ((u.spres >> d) & 1u)) ? uniform_u64(B.read_vc[(uint64_t)d * rstride + ridx]) : 0;
  };
  if (!GENERAL || !B.per_read_clock) load_clock(0, 1);

  // ---- batch metadata (lane i: read rb+i), double-buffered across batches ----
  struct Meta {
    uint64_t key, off0, off1, rb, r;  // rb: first slot of the batch; r: lane's read index
    uint64_t K;                       // packed view: the key's time base
    int32_t st;
    uint32_t nb, skip;  // skip: the row tier (am_rows.hip) owns this read
  };
  auto load_meta = [&](uint64_t bid, Meta &M) {
    M.rb = bid * WAVE;
    M.nb = bid < n_batches ? (uint32_t)(nsel - M.rb < (uint64_t)WAVE ? nsel - M.rb : (uint64_t)WAVE) : 0u;
    M.key = 0, M.off0 = 0, M.off1 = 0, M.st = AM_OK, M.r = 0, M.skip = 0, M.K = 0;
    if (lane < M.nb) {
      const uint64_t r = sbase ? (uint64_t)sbase[M.rb + lane] : M.rb + lane;
      M.r = r;
      const uint64_t key = B.key[r];
      const uint32_t rtype = B.type[r];
      M.key = key;
      if (key >= L.n_keys) {
        M.st = AM_ERR_INVALID;
      } else {
        M.off0 = L.key_off[key];
        M.off1 = am_kend(L, key);
        if (PACKED) M.K = L.key_tbase[key];
        const uint32_t ktype = L.key_type[key];
        const uint32_t kfl = L.key_flags ? (uint32_t)L.key_flags[key] : 0u;
        if (M.off1 > M.off0 && (ktype != rtype || (kfl & AM_KEY_MIXED_TYPES)))
          M.st = AM_ERR_CORRUPTED_OPS_CACHE;  // erlang:error(corrupted_ops_cache)
        else if (rtype != (uint32_t)TYPE)
          M.st = AM_ERR_INVALID;              // batch type_hint violated
      }
      if (M.st != AM_OK) M.off1 = M.off0;  // no tiles to stream
      if (H.mask && M.off1 - M.off0 <= (uint64_t)H.short_max) M.skip = 1, M.off1 = M.off0;
    }
    if (H.mask && bid < n_batches) {  // hand short (and error) reads to the row tier
      const uint64_t hm = __ballot(M.skip != 0);
      if (lane == 0) H.mask[bid] = hm;
    }
  };

  Acc<DMAX> a;
  AccP<DMAX> ap;
  PkRead<DMAX> pk;
  V v;
  a.reset();
  ap.reset();
  v.reset();
  Tile<DMAX> TA, TB;
  Out<DMAX> o;
  Meta M0, M1;

  // Per-lane buffered empty-log result (materialize/4 on []: FirstHole =
  // get_first_id([]) = 0, LastOpCt = the base snapshot_time, value = the base).
  // Every lane computes it for its own read; reads with ops overwrite it.
  auto init_out = [&](const Meta &M) {
    o.status = M.st;
    o.flags = 0, o.pres = 0, o.count = 0, o.ign = 1, o.newss = 0, o.nlo = 0, o.fin = 0;
#pragma unroll
    for (int d = 0; d < DMAX; ++d)
      if (BUF_CT) o.ct[d] = 0;
    o.v0 = 0, o.v1 = 0, o.vflag = TYPE == AM_LWW ? 1 : 0;
    if (GENERAL && lane < M.nb) {
      const uint64_t r = M.r;
      if (B.base_ignore && !B.base_ignore[r]) {
        o.ign = 0;
        o.pres = B.base_pres[r] & u.allmask;
#pragma unroll
        for (int d = 0; d < DMAX; ++d)
          if (BUF_CT && d < (int)nd && ((o.pres >> d) & 1u)) o.ct[d] = B.base_vc[(uint64_t)d * n + r];
      }
      if (B.base.v0) {
        o.v0 = (uint64_t)B.base.v0[r];
        if (TYPE == AM_LWW) {
          o.v1 = B.base.v1 ? B.base.v1[r] : 0;
          o.vflag = B.base.vflag ? B.base.vflag[r] : 0;
        }
      }
    }
  };
  // the batch's results: one coalesced store per column
  auto store_out = [&](const Meta &M) {
    if (lane < M.nb && !M.skip) {
      const uint64_t r = M.r;
      R.status[r] = o.status;
      if (o.status == AM_OK) {
        R.flags[r] = (uint8_t)o.flags;
        R.new_last_op[r] = o.nlo;
        R.last_ct_ignore[r] = (uint8_t)o.ign;
        R.last_ct_pres[r] = o.pres;
#pragma unroll
        for (int d = 0; d < DMAX; ++d) {
          if (d >= (int)nd) continue;
          if (BUF_CT) R.last_ct[(uint64_t)d * n + r] = o.ct[d];
          else if (!o.fin)  // no op streamed: LastOpCt = the base snapshot_time (finalize wrote the rest)
            R.last_ct[(uint64_t)d * n + r] = (GENERAL && ((o.pres >> d) & 1u)) ? B.base_vc[(uint64_t)d * n + r] : 0;
        }
        R.is_new_ss[r] = (uint8_t)o.newss;
        R.count[r] = o.count;
        R.value.v0[r] = (int64_t)o.v0;
        if (TYPE == AM_LWW) {
          R.value.v1[r] = o.v1;
          R.value.vflag[r] = (uint8_t)o.vflag;
        }
      }
    }
  };
  // first read (from j) of batch M that has a tile, or M.nb
  auto seek = [&](const Meta &M, uint32_t j, uint64_t &t) -> uint32_t {
    for (; j < M.nb; ++j) {
      const uint64_t o0 = lane_u64(M.off0, j), o1 = lane_u64(M.off1, j);
      if (o1 > o0) {
        t = o0 & ~(uint64_t)(OPL - 1);
        return j;
      }
    }
    return M.nb;
  };
  auto load_tile = [&](Tile<DMAX> &T, const Meta &M, uint32_t j, uint64_t t) {
    const uint64_t o1 = lane_u64(M.off1, j);
    const uint64_t g = t + (uint64_t)lane * OPL;
    T.meta4 = 0;
#pragma unroll
    for (int k = 0; k < OPL; ++k) {
      T.ct[k] = 0, T.p0[k] = 0, T.p1[k] = 0, T.tx[k] = 0, T.sp[k] = u.allmask;
#pragma unroll
      for (int d = 0; d < DMAX; ++d) T.sv[k][d] = 0, T.x[k][d] = 0;
    }
    if (g < o1 && PACKED) {
#pragma unroll
      for (int d = 0; d < DMAX; ++d) {
        if (d < (int)nd) {
          uint32_t xv[OPL];
          ld_u32<OPL>(L.pk_vc + (uint64_t)d * stride + g, xv);
#pragma unroll
          for (int k = 0; k < OPL; ++k) T.x[k][d] = xv[k];
        }
      }
    } else if (g < o1) {
      T.meta4 = OPL == 4 ? *(const uint32_t *)(L.op_meta + g) : (uint32_t)*(const uint16_t *)(L.op_meta + g);
      ld_u64<OPL>(L.commit_time + g, T.ct);
#pragma unroll
      for (int d = 0; d < DMAX; ++d) {
        if (d < (int)nd) {
          uint64_t svv[OPL];
          ld_u64<OPL>(L.snap_vc + (uint64_t)d * stride + g, svv);
#pragma unroll
          for (int k = 0; k < OPL; ++k) T.sv[k][d] = svv[k];
        }
      }
    }
    if (g < o1) {
      if (GENERAL && L.snap_pres) {
        ld_u32<OPL>(L.snap_pres + g, T.sp);
      }
      if (SOf<TYPE>::NEED_P0) ld_u64<OPL>(L.p0 + g, T.p0);
      if (SOf<TYPE>::NEED_P1) ld_u64<OPL>(L.p1 + g, T.p1);
      if (GENERAL && L.op_txid && B.txid) ld_u64<OPL>(L.op_txid + g, T.tx);
    }
  };
  auto setup_read = [&](uint32_t j) {  // per-read uniform inputs
    if (!GENERAL) {
      if (PACKED) pk_setup(u, nd, lane_u64(M0.K, j), pk);
      return;
    }
    const uint64_t r = lane_u64(M0.r, j);
    if (B.per_read_clock) load_clock(r, n);
    u.base_ignore = !B.base_ignore || B.base_ignore[r];
    u.cpres = u.base_ignore ? 0u : (uniform_u32(B.base_pres[r]) & u.allmask);
#pragma unroll
    for (int d = 0; d < DMAX; ++d)
      u.C0[d] = (d < (int)nd && ((u.cpres >> d) & 1u)) ? uniform_u64(B.base_vc[(uint64_t)d * n + r]) : 0;
    u.has_txid = B.txid && (!B.txid_valid || B.txid_valid[r]) && L.op_txid;
    u.txid = u.has_txid ? uniform_u64(B.txid[r]) : 0;
    if (PACKED) pk_setup(u, nd, lane_u64(M0.K, j), pk);
  };
  auto process = [&](const Tile<DMAX> &T, uint32_t j, uint64_t t) {
    const uint64_t o0 = lane_u64(M0.off0, j), o1 = lane_u64(M0.off1, j);
    const uint64_t g = t + (uint64_t)lane * OPL;
#pragma unroll
    for (int k = 0; k < OPL; ++k) {
      const uint64_t p = g + k;
      if (p < o0 || p >= o1) continue;
      const bool txm = GENERAL && u.has_txid && T.tx[k] == u.txid;
      if (PACKED) {
        if (T.x[k][0] == AM_PK_ESC) {  // rare: the op does not fit the packed view
          // (from the columns: the escape row's lookup here cost the batch-clock LWW kernel its
          // third wave per SIMD, 163 -> 169 VGPRs, and C2 1.55 -> 1.9 ms)
          uint64_t sv[DMAX];
#pragma unroll
          for (int d = 0; d < DMAX; ++d) sv[d] = d < (int)nd ? L.snap_vc[(uint64_t)d * stride + p] : 0;
          if (eval_op<DMAX, GENERAL>(u, L.op_meta[p], L.commit_time[p], sv, T.sp[k], txm, p, a)) v.add(T.p0[k], T.p1[k]);
        } else if (pk_eval<DMAX, GENERAL>(pk, u, T.x[k], txm, p, ap)) {
          v.add(T.p0[k], T.p1[k]);
        }
      } else if (eval_op<DMAX, GENERAL>(u, (T.meta4 >> (8 * k)) & 0xFFu, T.ct[k], T.sv[k], T.sp[k], txm, p, a)) {
        v.add(T.p0[k], T.p1[k]);
      }
    }
  };
  // Reduce read j of batch M0 across the wave and park its results in lane j.
  auto finalize = [&](uint32_t j) {
    const uint64_t key = lane_u64(M0.key, j);
    const uint64_t o0 = lane_u64(M0.off0, j), o1 = lane_u64(M0.off1, j);
    if (PACKED) pk_fold(ap, pk.K, u.allmask, a);
    const uint32_t count = wave_sum_u32(a.count);
    const uint32_t flags = wave_or_u32(a.flags);
    const uint32_t pres = wave_or_u32(a.pres);
    const uint64_t min_excl = wave_min_u64(a.min_excl);
    uint64_t mx[DMAX];
#pragma unroll
    for (int d = 0; d < DMAX; ++d) mx[d] = d < (int)nd ? wave_max_u64(a.mx[d]) : 0;
    int32_t status = (flags & FLAG_BAD) ? AM_ERR_UNEXPECTED_OPERATION : AM_OK;
    uint64_t v0 = 0, v1 = 0;
    uint32_t vflag = 0;
    if constexpr (TYPE == AM_PN) {
      int64_t hi = v.hi;
      uint64_t lo = v.lo;
      wave_sum_i128(hi, lo);
      const int64_t b = (GENERAL && B.base.v0) ? uniform_u64((uint64_t)B.base.v0[lane_u64(M0.r, j)]) : 0;
      add128(hi, lo, b < 0 ? -1 : 0, (uint64_t)b);
      if (status == AM_OK && hi != ((int64_t)lo < 0 ? -1 : 0)) status = AM_ERR_OVERFLOW;  // Erlang: bignum
      v0 = lo;
    } else if constexpr (TYPE == AM_LWW) {
      wave_max_lww(v);
      uint64_t bts = 0, bval = 0;
      uint32_t bbin = 1;  // new() = {0, <<>>}
      if (GENERAL && B.base.v0) {
        const uint64_t r = lane_u64(M0.r, j);
        bts = uniform_u64((uint64_t)B.base.v0[r]);
        bval = B.base.v1 ? uniform_u64(B.base.v1[r]) : 0;
        bbin = B.base.vflag ? uniform_u32(B.base.vflag[r]) : 0;
      }
      // erlang:max(Effect, State): the effect wins iff it sorts above the state
      const bool win = v.has && (v.ts > bts || (v.ts == bts && !bbin && v.val > bval));
      v0 = win ? v.ts : bts;
      v1 = win ? v.val : bval;
      vflag = win ? 0 : bbin;
    }
    // NewLastOp: id of the oldest excluded candidate - 1, else get_first_id/1
    const uint64_t idb = L.key_id_base ? uniform_u64(L.key_id_base[key]) : 1;
    int64_t nlo;
    if (min_excl != NONE)
      nlo = ((GENERAL && L.op_id) ? (int64_t)uniform_u64(L.op_id[min_excl]) : (int64_t)(idb + (min_excl - o0))) - 1;
    else
      nlo = (GENERAL && L.op_id) ? (int64_t)uniform_u64(L.op_id[o1 - 1]) : (int64_t)(idb + (o1 - o0) - 1);
    const bool ign = u.base_ignore && count == 0;
    const uint32_t opres = ign ? 0u : (pres | u.cpres);
    if (lane == j) {
      o.status = status;
      o.flags = flags & 0xFFu;
      o.count = count;
      o.pres = opres;
      o.ign = ign ? 1 : 0;
      o.newss = count > 0;
      o.nlo = nlo;
#pragma unroll
      for (int d = 0; d < DMAX; ++d) {
        const uint64_t m = mx[d] > u.C0[d] ? mx[d] : u.C0[d];
        if (BUF_CT) o.ct[d] = ((opres >> d) & 1u) ? m : 0;
      }
      o.v0 = v0, o.v1 = v1, o.vflag = vflag;
      o.fin = 1;
    }
    if (!BUF_CT && status == AM_OK) {  // wide clocks: lane d stores entry d of LastOpCt
      const uint64_t r = lane_u64(M0.r, j);
#pragma unroll
      for (int d = 0; d < DMAX; ++d) {
        const uint64_t m = mx[d] > u.C0[d] ? mx[d] : u.C0[d];
        if ((uint32_t)d == lane && d < (int)nd) R.last_ct[(uint64_t)d * n + r] = ((opres >> d) & 1u) ? m : 0;
      }
    }
    a.reset();
    ap.reset();
    v.reset();
  };
  // batch switch: M0's results leave, M1 becomes current, the next batch's metadata
  // is prefetched (it lands while the current batch streams)
  uint64_t bid = gw;
  auto switch_batch = [&]() {
    store_out(M0);
    M0 = M1;
    bid += W;
    init_out(M0);
    load_meta(bid + W, M1);
  };

  load_meta(bid, M0);
  load_meta(bid + W, M1);
  init_out(M0);
  while (bid < n_batches) {
    // ---- one double-buffered tile stream; it runs on into the next batch(es) ----
    uint64_t ct_ = 0;
    uint32_t cj = seek(M0, 0, ct_);
    if (cj >= M0.nb) {  // no tile in this batch
      switch_batch();
      continue;
    }
    bool first = true;
    load_tile(TA, M0, cj, ct_);
    // One pipeline step: issue the next tile's loads, then consume `cur`.
    auto step = [&](Tile<DMAX> &cur, Tile<DMAX> &nxt) -> bool {
      uint64_t nt = ct_ + TILE;
      uint32_t nj = cj;
      bool cross = false;
      if (nt >= lane_u64(M0.off1, cj)) {
        nj = seek(M0, cj + 1, nt);
        if (nj >= M0.nb) {  // the next tile belongs to the next batch (if any)
          nj = seek(M1, 0, nt);
          cross = true;
        }
      }
      const bool more = cross ? nj < M1.nb : true;
      if (more) load_tile(nxt, cross ? M1 : M0, nj, nt);
      if (first) setup_read(cj);
      process(cur, cj, ct_);
      first = cross || nj != cj;
      if (first) finalize(cj);
      if (cross && more) switch_batch();
      cj = nj;
      ct_ = nt;
      return more;
    };
    while (true) {
      if (!step(TA, TB)) break;
      if (!step(TB, TA)) break;
    }
    switch_batch();  // the stream ended inside M0 (M1 has no tile or does not exist)
  }
}

}  // namespace amk_stream
