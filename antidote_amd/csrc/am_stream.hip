// am_stream.hip -- the streaming materialize kernel (default path).
//
// Work split: each wavefront owns a contiguous range of reads.  It loads the
// metadata of 64 reads at a time with one vector load per lane (lane i: read
// mb+i -> key, key_off[key], key_off[key+1], key_type), so no per-read
// dependent global load sits on the critical path; the current read's metadata
// is broadcast with v_readlane.  The wave then walks the reads' op logs as one
// stream of 256-op tiles (lane l owns 4 consecutive ops of a tile: 16-byte
// loads, one contiguous 2 KiB segment per u64 column per wave instruction) and
// DOUBLE-BUFFERS it: the next tile's loads (possibly the next read's first tile)
// are issued before the current tile is evaluated, reduced (DPP row butterflies
// + 4 readlanes) and its read's outputs stored, so the wave keeps a tile of HBM
// traffic in flight through its whole lifetime.
//
// Semantics per op / per read: see am_wave.h (eval_op) and am_materialize.hip.
#include "am_wave.h"

using namespace amk;

namespace {

constexpr int BLOCK = 256;
constexpr int WPB = BLOCK / WAVE;
constexpr int OPL = 4;
constexpr uint64_t TILE = WAVE * OPL;

template <int DMAX>
struct Tile {
  uint32_t meta4;
  uint64_t ct[OPL];
  uint64_t sv[OPL][DMAX];
  uint32_t sp[OPL];
  uint64_t p0[OPL], p1[OPL], tx[OPL];
};

// status codes kept in the per-lane metadata word (bits 0..7 = am_status + 16)
__device__ __forceinline__ uint32_t enc_status(int s) { return (uint32_t)(s + 16) & 0xFFu; }
__device__ __forceinline__ int dec_status(uint32_t w) { return (int)(w & 0xFFu) - 16; }

template <int DMAX, int TYPE, bool GENERAL>
__global__ void __launch_bounds__(BLOCK) k_stream(am_op_log L, am_read_batch B, am_read_result R, int INTERLEAVE) {
  using V = typename ValOf<TYPE>::T;
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  const uint64_t n = B.n_reads;
  const uint32_t nd = L.n_dc;
  const uint64_t stride = L.snap_stride ? L.snap_stride : L.n_ops;
  const uint64_t W = (uint64_t)gridDim.x * WPB;
  const uint64_t gw = (uint64_t)blockIdx.x * WPB + uniform_u32(threadIdx.x >> 6);
  // Read ordinal k of this wave -> read index.  Interleaved (default): wave gw owns
  // reads gw, gw+W, gw+2W, ... so at any moment the grid streams ADJACENT keys'
  // logs (a few DRAM pages per column); contiguous: gw owns one block of reads.
  const uint64_t per = (n + W - 1) / W;
  const uint64_t cnt = INTERLEAVE ? (n > gw ? (n - gw + W - 1) / W : 0)
                                  : (gw * per < n ? ((gw + 1) * per < n ? per : n - gw * per) : 0);
  auto rid = [&](uint64_t k) -> uint64_t { return INTERLEAVE ? gw + k * W : gw * per + k; };
  if (cnt == 0) return;

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

  Acc<DMAX> a;
  V v;
  a.reset();
  v.reset();
  Tile<DMAX> TA, TB;

  for (uint64_t kb = 0; kb < cnt; kb += WAVE) {
    const uint32_t nb = (uint32_t)(cnt - kb < (uint64_t)WAVE ? cnt - kb : (uint64_t)WAVE);
    // ---- metadata of this wave's reads kb .. kb+nb-1, one per lane ----
    uint64_t m_key = 0, m_off0 = 0, m_off1 = 0;
    uint32_t m_info = enc_status(AM_OK);
    if (lane < nb) {
      const uint64_t r = rid(kb + lane);
      const uint64_t key = B.key[r];
      const uint32_t rtype = B.type[r];
      m_key = key;
      if (key >= L.n_keys) {
        m_info = enc_status(AM_ERR_INVALID);
      } else {
        m_off0 = L.key_off[key];
        m_off1 = L.key_off[key + 1];
        const uint32_t ktype = L.key_type[key];
        const uint32_t kfl = L.key_flags ? (uint32_t)L.key_flags[key] : 0u;
        if (m_off1 > m_off0 && (ktype != rtype || (kfl & AM_KEY_MIXED_TYPES)))
          m_info = enc_status(AM_ERR_CORRUPTED_OPS_CACHE);  // erlang:error(corrupted_ops_cache)
        else if (rtype != (uint32_t)TYPE)
          m_info = enc_status(AM_ERR_INVALID);               // batch type_hint violated
      }
      if (dec_status(m_info) != AM_OK) m_off1 = m_off0;      // no tiles to stream
    }

    // Emit a read that streams no tile (no ops, or an error status).
    auto emit_notile = [&](uint32_t j) {
      const uint64_t r = rid(kb + j);
      const int st = dec_status(lane_u32(m_info, j));
      if (lane != 0) return;
      R.status[r] = st;
      if (st != AM_OK) return;
      R.flags[r] = 0;
      // materialize/4 with an empty ops list: FirstHole = get_first_id([]) = 0,
      // LastOpCt = the base snapshot_time, value = the base value
      R.new_last_op[r] = 0;
      R.is_new_ss[r] = 0;
      R.count[r] = 0;
      bool bign = true;
      uint32_t cp = 0;
      if (GENERAL && B.base_ignore && !B.base_ignore[r]) {
        bign = false;
        cp = B.base_pres[r] & u.allmask;
      }
      R.last_ct_ignore[r] = bign ? 1 : 0;
      R.last_ct_pres[r] = cp;
      for (uint32_t d = 0; d < nd; ++d) R.last_ct[(uint64_t)d * n + r] = ((cp >> d) & 1u) ? B.base_vc[(uint64_t)d * n + r] : 0;
      if constexpr (TYPE == AM_PN) {
        R.value.v0[r] = (GENERAL && B.base.v0) ? B.base.v0[r] : 0;
      } else {
        const bool hb = GENERAL && B.base.v0;
        R.value.v0[r] = hb ? B.base.v0[r] : 0;
        R.value.v1[r] = hb && B.base.v1 ? B.base.v1[r] : 0;
        R.value.vflag[r] = hb ? (B.base.vflag ? B.base.vflag[r] : 0) : 1;
      }
    };
    auto tiles_of = [&](uint32_t j, uint64_t &t0, uint64_t &o0, uint64_t &o1) {
      o0 = lane_u64(m_off0, j);
      o1 = lane_u64(m_off1, j);
      t0 = o0 & ~(uint64_t)(OPL - 1);
    };
    // advance to the first read (from j) that has a tile; reads skipped are emitted
    auto seek = [&](uint32_t j, uint64_t &t) -> uint32_t {
      for (; j < nb; ++j) {
        uint64_t t0, o0, o1;
        tiles_of(j, t0, o0, o1);
        if (o1 > o0) {
          t = t0;
          return j;
        }
        emit_notile(j);
      }
      return nb;
    };
    auto load_tile = [&](Tile<DMAX> &T, uint32_t j, uint64_t t) {
      const uint64_t o1 = lane_u64(m_off1, j);
      const uint64_t g = t + (uint64_t)lane * OPL;
      const bool live = g < o1;
      T.meta4 = 0;
#pragma unroll
      for (int k = 0; k < OPL; ++k) {
        T.ct[k] = 0, T.p0[k] = 0, T.p1[k] = 0, T.tx[k] = 0, T.sp[k] = u.allmask;
#pragma unroll
        for (int d = 0; d < DMAX; ++d) T.sv[k][d] = 0;
      }
      if (live) {
        T.meta4 = *(const uint32_t *)(L.op_meta + g);
        const u64x2 c01 = *(const u64x2 *)(L.commit_time + g), c23 = *(const u64x2 *)(L.commit_time + g + 2);
        T.ct[0] = c01.x, T.ct[1] = c01.y, T.ct[2] = c23.x, T.ct[3] = c23.y;
#pragma unroll
        for (int d = 0; d < DMAX; ++d) {
          if (d < (int)nd) {
            const uint64_t *col = L.snap_vc + (uint64_t)d * stride + g;
            const u64x2 s01 = *(const u64x2 *)col, s23 = *(const u64x2 *)(col + 2);
            T.sv[0][d] = s01.x, T.sv[1][d] = s01.y, T.sv[2][d] = s23.x, T.sv[3][d] = s23.y;
          }
        }
        if (GENERAL && L.snap_pres) {
          const u32x4 s = *(const u32x4 *)(L.snap_pres + g);
          T.sp[0] = s.x, T.sp[1] = s.y, T.sp[2] = s.z, T.sp[3] = s.w;
        }
        const u64x2 a01 = *(const u64x2 *)(L.p0 + g), a23 = *(const u64x2 *)(L.p0 + g + 2);
        T.p0[0] = a01.x, T.p0[1] = a01.y, T.p0[2] = a23.x, T.p0[3] = a23.y;
        if (ValOf<TYPE>::NEED_P1) {
          const u64x2 b01 = *(const u64x2 *)(L.p1 + g), b23 = *(const u64x2 *)(L.p1 + g + 2);
          T.p1[0] = b01.x, T.p1[1] = b01.y, T.p1[2] = b23.x, T.p1[3] = b23.y;
        }
        if (GENERAL && L.op_txid && B.txid) {
          const u64x2 x01 = *(const u64x2 *)(L.op_txid + g), x23 = *(const u64x2 *)(L.op_txid + g + 2);
          T.tx[0] = x01.x, T.tx[1] = x01.y, T.tx[2] = x23.x, T.tx[3] = x23.y;
        }
      }
    };
    auto setup_read = [&](uint32_t j) {  // per-read uniform inputs (GENERAL only)
      if (!GENERAL) return;
      const uint64_t r = rid(kb + j);
      if (B.per_read_clock) load_clock(r, n);
      u.base_ignore = !B.base_ignore || B.base_ignore[r];
      u.cpres = u.base_ignore ? 0u : (uniform_u32(B.base_pres[r]) & u.allmask);
#pragma unroll
      for (int d = 0; d < DMAX; ++d)
        u.C0[d] = (d < (int)nd && ((u.cpres >> d) & 1u)) ? uniform_u64(B.base_vc[(uint64_t)d * n + r]) : 0;
      u.has_txid = B.txid && (!B.txid_valid || B.txid_valid[r]) && L.op_txid;
      u.txid = u.has_txid ? uniform_u64(B.txid[r]) : 0;
    };
    auto process = [&](const Tile<DMAX> &T, uint32_t j, uint64_t t) {
      const uint64_t o0 = lane_u64(m_off0, j), o1 = lane_u64(m_off1, j);
      const uint64_t g = t + (uint64_t)lane * OPL;
#pragma unroll
      for (int k = 0; k < OPL; ++k) {
        const uint64_t p = g + k;
        if (p < o0 || p >= o1) continue;
        const bool txm = GENERAL && u.has_txid && T.tx[k] == u.txid;
        if (eval_op<DMAX, GENERAL>(u, (T.meta4 >> (8 * k)) & 0xFFu, T.ct[k], T.sv[k], T.sp[k], txm, p, a))
          v.add(T.p0[k], T.p1[k]);
      }
    };
    auto finalize = [&](uint32_t j) {
      const uint64_t r = rid(kb + j);
      const uint64_t key = lane_u64(m_key, j);
      const uint64_t o0 = lane_u64(m_off0, j), o1 = lane_u64(m_off1, j);
      const uint32_t count = wave_sum_u32(a.count);
      const uint32_t flags = wave_or_u32(a.flags);
      const uint64_t min_excl = wave_min_u64(a.min_excl);
      uint64_t mx[DMAX];
#pragma unroll
      for (int d = 0; d < DMAX; ++d) mx[d] = d < (int)nd ? wave_max_u64(a.mx[d]) : 0;
      const uint32_t pres = wave_or_u32(a.pres);
      int32_t status = (flags & FLAG_BAD) ? AM_ERR_UNEXPECTED_OPERATION : AM_OK;
      if constexpr (TYPE == AM_PN) {
        int64_t hi = v.hi;
        uint64_t lo = v.lo;
        wave_sum_i128(hi, lo);
        if (lane == 0 && status == AM_OK) {
          const int64_t b = (GENERAL && B.base.v0) ? B.base.v0[r] : 0;
          add128(hi, lo, b < 0 ? -1 : 0, (uint64_t)b);
          if (hi != ((int64_t)lo < 0 ? -1 : 0))
            status = AM_ERR_OVERFLOW;  // Erlang would return a bignum
          else
            R.value.v0[r] = (int64_t)lo;
        }
      } else {
        wave_max_lww(v);
        if (lane == 0 && status == AM_OK) {
          uint64_t bts = 0, bval = 0;
          uint32_t bbin = 1;  // new() = {0, <<>>}
          if (GENERAL && B.base.v0) {
            bts = (uint64_t)B.base.v0[r];
            bval = B.base.v1 ? B.base.v1[r] : 0;
            bbin = B.base.vflag ? B.base.vflag[r] : 0;
          }
          const bool win = v.has && (v.ts > bts || (v.ts == bts && !bbin && v.val > bval));
          R.value.v0[r] = (int64_t)(win ? v.ts : bts);
          R.value.v1[r] = win ? v.val : bval;
          R.value.vflag[r] = win ? 0 : (uint8_t)bbin;
        }
      }
      if (lane == 0) {
        R.status[r] = status;
        R.flags[r] = (uint8_t)(flags & 0xFFu);
        if (status == AM_OK) {
          const uint64_t idb = L.key_id_base ? L.key_id_base[key] : 1;
          const uint64_t nops = o1 - o0;
          int64_t nlo;
          if (min_excl != NONE)
            nlo = ((GENERAL && L.op_id) ? (int64_t)L.op_id[min_excl] : (int64_t)(idb + (min_excl - o0))) - 1;
          else
            nlo = (GENERAL && L.op_id) ? (int64_t)L.op_id[o1 - 1] : (int64_t)(idb + nops - 1);
          R.new_last_op[r] = nlo;
          const bool ign = u.base_ignore && count == 0;
          const uint32_t opres = ign ? 0u : (pres | u.cpres);
          R.last_ct_ignore[r] = ign ? 1 : 0;
          R.last_ct_pres[r] = opres;
#pragma unroll
          for (int d = 0; d < DMAX; ++d) {
            if (d < (int)nd) {
              const uint64_t m = mx[d] > u.C0[d] ? mx[d] : u.C0[d];
              R.last_ct[(uint64_t)d * n + r] = ((opres >> d) & 1u) ? m : 0;
            }
          }
          R.is_new_ss[r] = count > 0;
          R.count[r] = count;
        }
      }
      a.reset();
      v.reset();
    };

    // ---- double-buffered tile stream over the batch ----
    uint64_t ct_ = 0;
    uint32_t cj = seek(0, ct_);
    if (cj >= nb) continue;
    bool first = true;
    load_tile(TA, cj, ct_);
    // One pipeline step: issue the next tile's loads, then consume `cur`.
    auto step = [&](Tile<DMAX> &cur, Tile<DMAX> &nxt) -> bool {
      uint64_t nt = ct_ + TILE;
      uint32_t nj = cj;
      const uint64_t o1 = lane_u64(m_off1, cj);
      if (nt >= o1) nj = seek(cj + 1, nt);
      const bool more = nj < nb;
      if (more) load_tile(nxt, nj, nt);
      if (first) setup_read(cj);
      process(cur, cj, ct_);
      first = nj != cj;
      if (first) finalize(cj);
      cj = nj;
      ct_ = nt;
      return more;
    };
    while (true) {
      if (!step(TA, TB)) break;
      if (!step(TB, TA)) break;
    }
  }
}

template <int TYPE, bool GENERAL>
int launch(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R) {
  // persistent-style grid: exactly the resident capacity (every wave streams one
  // contiguous range of reads for the kernel's whole lifetime), never more blocks
  // than 4 reads per block
  static int occ[3][8] = {};
  const uint32_t nd = L->n_dc;
  const int di = nd <= 1 ? 0 : nd <= 2 ? 1 : nd <= 3 ? 2 : nd <= 4 ? 3 : nd <= 8 ? 4 : nd <= 16 ? 5 : 6;
  int &o = occ[TYPE][di];
  if (o == 0) {
    int nb = 0;
    hipError_t e = hipErrorInvalidValue;
    switch (di) {
      case 0: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_stream<1, TYPE, GENERAL>, BLOCK, 0); break;
      case 1: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_stream<2, TYPE, GENERAL>, BLOCK, 0); break;
      case 2: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_stream<3, TYPE, GENERAL>, BLOCK, 0); break;
      case 3: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_stream<4, TYPE, GENERAL>, BLOCK, 0); break;
      case 4: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_stream<8, TYPE, GENERAL>, BLOCK, 0); break;
      case 5: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_stream<16, TYPE, GENERAL>, BLOCK, 0); break;
      default: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_stream<32, TYPE, GENERAL>, BLOCK, 0); break;
    }
    o = (e == hipSuccess && nb > 0) ? nb : 2;
  }
  uint64_t blocks = (B->n_reads + WPB - 1) / WPB;
  const uint64_t cap = (uint64_t)ctx->n_cu * (uint64_t)o;
  if (blocks > cap) blocks = cap;
  if (blocks == 0) return AM_OK;
  dim3 grid((unsigned)blocks), block(BLOCK);
  const char *iv = getenv("AM_INTERLEAVE");
  const int inter = iv ? atoi(iv) : 1;
#define AM_L(D)                                                                                  \
  hipLaunchKernelGGL((k_stream<D, TYPE, GENERAL>), grid, block, 0, ctx->stream, *L, *B, *R, inter); \
  break;
  switch (nd <= 1 ? 1 : nd <= 2 ? 2 : nd <= 3 ? 3 : nd <= 4 ? 4 : nd <= 8 ? 8 : nd <= 16 ? 16 : 32) {
    case 1: AM_L(1)
    case 2: AM_L(2)
    case 3: AM_L(3)
    case 4: AM_L(4)
    case 8: AM_L(8)
    case 16: AM_L(16)
    default: AM_L(32)
  }
#undef AM_L
  AM_HIP(hipGetLastError());
  return AM_OK;
}

}  // namespace

// FAST variant when the batch uses none of: partial snapshot clocks, explicit op
// ids, TxIds, cached bases, per-read clocks (the bench's fresh snapshot read).
int am_launch_stream(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R) {
  const bool general = L->snap_pres || L->op_id || (B->txid && L->op_txid) || B->base_ignore || B->per_read_clock ||
                       B->base.v0;
  switch (B->type_hint) {
    case AM_PN: return general ? launch<AM_PN, true>(ctx, L, B, R) : launch<AM_PN, false>(ctx, L, B, R);
    case AM_LWW: return general ? launch<AM_LWW, true>(ctx, L, B, R) : launch<AM_LWW, false>(ctx, L, B, R);
    default:
      return AM_ERR_UNSUPPORTED;
  }
}
