// am_lanes.hip -- materialize/4 for SHORT logs, one LANE per read, PN counter, LWW register,
// add-wins set and MV register reads in ONE launch.
//
// Most of a partition's keys are short (the mixed C4 workload: 16 ops per key; C5: 95 % of
// keys with <= 48 ops).  A 16-lane row per read (am_rows.hip) keeps only 4 reads of a wave in
// flight, each lane holding one 4-byte entry per column, and pays a row reduction per read;
// per-type launches over a type-mixed log also re-fetch the cache lines that neighbouring keys
// of the other types share.  Here lane i of a wave owns read i of a 64-read batch outright:
//   * the read's ops stream in OPL-op tiles (16-byte loads of the packed view, payload words
//     with them for PN / LWW; is_op_in_snapshot/7 on u32 entries, am_group.h pk_tile);
//     inclusion bits in a u64;
//   * PN: exact 128-bit sum; LWW: erlang:max on {Ts, Value} (am_wave.h PnVal / LwwVal);
//   * AW / MV: the key's token-group records (am_group.h) set born / killed bits of at most
//     64 groups in two u64 registers; survivors = born & ~killed, gathered in group order
//     (already the reference's output order);
//   * no cross-lane reduction: every output column leaves with one coalesced store per batch.
// A read the kernel does not take (a longer log, more groups, an ungrouped key, base-snapshot
// pairs, a bounded counter, a type outside `accept`) goes to `next`; reads with an unknown
// key or type, or a corrupted ops cache (src/clocksi_materializer.erl:190-191), get their
// status here.
#include "am_group.h"

using namespace amk;
using namespace amk_grp;

namespace {

constexpr uint32_t LBITS = 64;  // inclusion bits of a lane read: ops [off0 & ~(OPL-1), off1)
constexpr uint32_t LGRP = 64;   // groups of a lane set read (u64 born / killed)
constexpr int LBLOCK = 256;
// ops per lane tile: two 16-byte loads per packed column at D <= 8 (each lane's loads of a
// 64-byte segment issued back to back measured 6-8 % faster on C4 than a double-buffered
// 4-op tile, and 3-9 % faster than 16-op tiles or higher occupancy); D > 8: 4
template <int DMAX>
constexpr int lopl() {
  return DMAX <= 8 ? 8 : 4;
}

// ---- quad all-reductions (DPP quad_perm 1032, 2301): every lane of a quad ends with the
// quad's value.  All 64 lanes must be active (DPP reads an inactive lane as 0).
__device__ __forceinline__ uint32_t quad_or_u32(uint32_t v) {
  v |= dpp32<0xB1>(v);
  return v | dpp32<0x4E>(v);
}
__device__ __forceinline__ uint64_t quad_or_u64(uint64_t v) {
  v |= dpp64<0xB1>(v);
  return v | dpp64<0x4E>(v);
}
__device__ __forceinline__ uint32_t quad_sum_u32(uint32_t v) {
  v += dpp32<0xB1>(v);
  return v + dpp32<0x4E>(v);
}
__device__ __forceinline__ uint32_t quad_max_u32(uint32_t v) {
  v = max(v, dpp32<0xB1>(v));
  return max(v, dpp32<0x4E>(v));
}
__device__ __forceinline__ uint32_t quad_min_u32(uint32_t v) {
  v = min(v, dpp32<0xB1>(v));
  return min(v, dpp32<0x4E>(v));
}
__device__ __forceinline__ uint64_t quad_min_u64(uint64_t v) {
  v = umin64(v, dpp64<0xB1>(v));
  return umin64(v, dpp64<0x4E>(v));
}
template <int C>
__device__ __forceinline__ void quad_step_i128(int64_t &hi, uint64_t &lo) {
  const uint64_t wlo = dpp64<C>(lo);
  const int64_t whi = (int64_t)dpp64<C>((uint64_t)hi);
  add128(hi, lo, whi, wlo);
}
template <int C>
__device__ __forceinline__ void quad_step_lww(LwwVal &v) {
  const uint64_t ts = dpp64<C>(v.ts), val = dpp64<C>(v.val);
  const uint32_t has = dpp32<C>(v.has);
  const bool gt = has && (!v.has || ts > v.ts || (ts == v.ts && val > v.val));
  v.ts = gt ? ts : v.ts;
  v.val = gt ? val : v.val;
  v.has |= has;
}

// position of the k-th (0-based) set bit of m (k < popcount(m))
__device__ __forceinline__ uint32_t select64(uint64_t m, uint32_t k) {
  uint32_t pos = 0, c = (uint32_t)__popc((uint32_t)m);
  if (k >= c) k -= c, m >>= 32, pos += 32;
  c = (uint32_t)__popc((uint32_t)m & 0xFFFFu);
  if (k >= c) k -= c, m >>= 16, pos += 16;
  c = (uint32_t)__popc((uint32_t)m & 0xFFu);
  if (k >= c) k -= c, m >>= 8, pos += 8;
  c = (uint32_t)__popc((uint32_t)m & 0xFu);
  if (k >= c) k -= c, m >>= 4, pos += 4;
  c = (uint32_t)__popc((uint32_t)m & 0x3u);
  if (k >= c) k -= c, m >>= 2, pos += 2;
  return pos + (k >= ((uint32_t)m & 1u) ? 1u : 0u);
}

// The wave's survivor gather: lane l contributes n survivors (alive bits of its read's groups,
// pairs at grp[2 (src + g)], output slots dst, dst + 1, ...).  Entry j of the wave's list is
// taken by lane j % 64: its owner is the last lane whose exclusive prefix is <= j, its group the
// (j - prefix)-th set bit of the owner's mask.  All 64 lanes must be active.
__device__ __forceinline__ void wave_gather(const am_op_log &L, const am_read_result &R, uint32_t n, uint64_t alive,
                                            uint64_t src, uint64_t dst, uint32_t lane) {
  const uint32_t incl = wave_incl_scan_u32(n, lane), excl = incl - n;
  const uint32_t T = lane_u32(incl, WAVE - 1);
  constexpr int K = 4;
  for (uint32_t base = 0; base < T; base += K * WAVE) {
    u64x2 ab[K];
    uint64_t to[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const uint32_t j = base + (uint32_t)k * WAVE + lane;
      const uint32_t jj = j < T ? j : T - 1;
      uint32_t own = 0;
#pragma unroll
      for (uint32_t step = 32; step; step >>= 1) {
        const uint32_t c = own + step;
        if (c < (uint32_t)WAVE && shfl_u32(excl, c) <= jj) own = c;
      }
      const uint32_t rank = jj - shfl_u32(excl, own);
      const uint64_t m = shfl_u64(alive, own), s0 = shfl_u64(src, own), d0 = shfl_u64(dst, own);
      to[k] = j < T ? d0 + rank : ~0ull;
      if (j < T) ab[k] = *(const u64x2 *)(L.grp + 2 * (s0 + select64(m, rank)));
    }
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (to[k] != ~0ull) R.value.set_a[to[k]] = ab[k].x, R.value.set_b[to[k]] = ab[k].y;
  }
}

// four records [q, q + 4) of a set read with records [rk0, rk1): an included op's birth sets
// its group's born bit, its effective kill the killed bit (incl bit = op index + sh)
__device__ __forceinline__ void rec_bits(u32x4 v, uint64_t q, uint64_t rk0, uint64_t rk1, uint64_t incl, uint32_t sh,
                                         uint64_t &born, uint64_t &killed) {
  const uint32_t xs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t x = xs[k];
    if (q + k < rk0 || q + k >= rk1 || x == 0xFFFFFFFFu) continue;
    if (!((incl >> (AM_REC_OP(x) + sh)) & 1ull)) continue;
    const uint64_t bit = 1ull << AM_REC_GRP(x);
    if (x & AM_REC_KILL) killed |= bit;
    else born |= bit;
  }
}

// a lane read's outputs (materialize/4's {ok, Value, NewLastOp, LastOpCt, IsNewSS, Count} or
// its error status): one coalesced store per column over the wave
template <int DMAX>
__device__ __forceinline__ void write_lane(const am_op_log &L, const am_read_result &R, const ReadU<DMAX> &u,
                                           uint32_t nd, uint64_t n, uint64_t r, uint64_t idb, uint64_t off0,
                                           uint64_t off1, uint32_t t, int32_t status, const Acc<DMAX> &a, uint64_t v0,
                                           uint64_t v1, uint32_t vflag, uint32_t ns) {
  R.status[r] = status;
  R.flags[r] = (uint8_t)(a.flags & 0xFFu);
  if (status != AM_OK) return;
  R.new_last_op[r] = new_last_op_b(L, idb, off0, off1, a.min_excl);
  const bool ign = u.base_ignore && a.count == 0;
  const uint32_t opres = ign ? 0u : (a.pres | u.cpres);
  R.last_ct_ignore[r] = ign ? 1 : 0;
  R.last_ct_pres[r] = opres;
#pragma unroll
  for (int d = 0; d < DMAX; ++d) {
    if (d >= (int)nd) continue;
    const uint64_t m = a.mx[d] > u.C0[d] ? a.mx[d] : u.C0[d];
    R.last_ct[(uint64_t)d * n + r] = ((opres >> d) & 1u) ? m : 0;
  }
  R.is_new_ss[r] = a.count > 0;
  R.count[r] = a.count;
  if (t == AM_PN || t == AM_LWW) R.value.v0[r] = (int64_t)v0;
  if (t == AM_LWW) {
    R.value.v1[r] = v1;
    R.value.vflag[r] = (uint8_t)vflag;
  }
  if (t == AM_AWSET || t == AM_MVREG) R.value.set_len[r] = ns;
}

// ================================================================ general reads
// Per-read clocks, cached bases, TxIds or op ids: one lane walks its read's ops in OPL-op tiles.
template <int DMAX, int OPL>
struct LTile {
  uint32_t x[OPL][DMAX];
  uint64_t tx[OPL];
  uint64_t v0[OPL], v1[OPL];
};

template <int DMAX>
__global__ void __launch_bounds__(LBLOCK) k_lane_g(am_op_log L, am_read_batch B, am_read_result R, am_sel S,
                                                   am_retry next, uint32_t accept) {
  constexpr int OPL = lopl<DMAX>();
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  const uint64_t lt = (1ull << lane) - 1ull;
  const uint32_t nd = L.n_dc;
  const uint64_t stride = L.snap_stride ? L.snap_stride : L.n_ops;
  const uint32_t sel0 = S.idx ? uniform_u32(S.range[0]) : 0u;
  const uint64_t nsel = S.idx ? (uint64_t)(uniform_u32(S.range[1]) - sel0) : B.n_reads;
  const uint64_t n = B.n_reads;
  ReadU<DMAX> u{};

  const uint64_t step = (uint64_t)gridDim.x * LBLOCK;
  for (uint64_t b0 = (uint64_t)blockIdx.x * LBLOCK + (threadIdx.x & ~(WAVE - 1)); b0 < nsel; b0 += step) {
    const uint64_t i = b0 + lane;
    uint64_t r = 0, key = 0, off0 = 0, off1 = 0, rk0 = 0, rk1 = 0;
    uint32_t t = 0, G = 0;
    int32_t st = AM_OK;
    bool take = false, hand = false;
    if (i < nsel) {
      r = S.idx ? (uint64_t)S.idx[sel0 + i] : i;
      key = B.key[r];
      t = B.type[r];
      if (key >= L.n_keys || t < AM_PN || t > AM_BCOUNTER) {
        st = AM_ERR_INVALID;
      } else {
        off0 = L.key_off[key];
        off1 = am_kend(L, key);
        const uint32_t ktype = L.key_type[key];
        const uint32_t kfl = L.key_flags ? (uint32_t)L.key_flags[key] : 0u;
        if (off1 > off0 && (ktype != t || (kfl & AM_KEY_MIXED_TYPES))) st = AM_ERR_CORRUPTED_OPS_CACHE;
      }
      if (st == AM_OK) {
        bool ok = ((accept >> t) & 1u) && off1 - (off0 & ~(uint64_t)(OPL - 1)) <= LBITS;
        if (ok && (t == AM_AWSET || t == AM_MVREG)) {
          G = L.key_ngrp[key];
          rk0 = L.rec_key_off[key];
          rk1 = am_rkend(L, key);
          ok = G != AM_NGRP_NONE && G <= LGRP && !has_base_pairs(B, r);
        }
        take = ok;
        hand = !ok;
      } else {
        R.status[r] = st;
        R.flags[r] = 0;
      }
    }
    const uint64_t hm = __ballot(hand);
    if (hm) {
      uint32_t base = 0;
      if (lane == 0) base = atomicAdd(next.count, (uint32_t)__popcll(hm));
      base = uniform_u32(base);
      if (hand) next.list[base + (uint32_t)__popcll(hm & lt)] = (uint32_t)r;
    }
    if (!__ballot(take)) continue;

    // ---- this lane's read ----
    const bool scal = t == AM_PN || t == AM_LWW, setr = t == AM_AWSET || t == AM_MVREG;
    if (take) read_inputs<DMAX, true, false>(L, nd, B, r, u);
    PkRead<DMAX> pk;
    pk_setup(u, nd, take ? L.key_tbase[key] : 0, pk);
    const uint64_t t0 = off0 & ~(uint64_t)(OPL - 1);
    const uint32_t sh = (uint32_t)(off0 - t0);
    // the first record vector of a set read is in flight with the ops
    const uint64_t q0 = rk0 & ~3ull;
    u32x4 rv = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    if (take && setr && rk1 > rk0) rv = *(const u32x4 *)(L.rec_g + q0);

    AccP<DMAX> ap;
    Acc<DMAX> a;
    ap.reset();
    a.reset();
    PnVal pv;
    LwwVal lv;
    pv.reset();
    lv.reset();
    bool esc = false;
    uint64_t incl = 0;
    LTile<DMAX, OPL> cur;
    for (uint64_t g = t0; take && g < off1; g += OPL) {
#pragma unroll
      for (int d = 0; d < DMAX; ++d) {
        uint32_t q[OPL] = {};
        if (d < (int)nd) ld_n32<OPL>(L.pk_vc + (uint64_t)d * stride + g, q);
#pragma unroll
        for (int k = 0; k < OPL; ++k) cur.x[k][d] = q[k];
      }
#pragma unroll
      for (int k = 0; k < OPL; ++k) cur.tx[k] = 0, cur.v0[k] = 0, cur.v1[k] = 0;
      if (u.has_txid) ld_n64<OPL>(L.op_txid + g, cur.tx);
      if (scal) ld_n64<OPL>(L.p0 + g, cur.v0);
      if (t == AM_LWW) ld_n64<OPL>(L.p1 + g, cur.v1);
      const uint32_t ib = pk_tile<DMAX, OPL, true>(u, pk, cur.x, cur.tx, g, off0, off1, ap, esc);
      incl |= (uint64_t)ib << (g - t0);
      if (scal) {
#pragma unroll
        for (int k = 0; k < OPL; ++k)
          if ((ib >> k) & 1u) {
            if (t == AM_PN) pv.add(cur.v0[k], 0);
            else lv.add(cur.v0[k], cur.v1[k]);
          }
      }
    }
    if (esc) {  // rare: ops outside the packed view, from the full columns
      for (uint64_t p = off0; p < off1; ++p) {
        if (L.pk_vc[p] != AM_PK_ESC) continue;
        uint64_t sv[DMAX], ct;
        uint32_t meta;
        esc_load<DMAX>(L, nd, stride, p, sv, ct, meta);
        const uint32_t sp = L.snap_pres ? L.snap_pres[p] : u.allmask;
        const bool txm = u.has_txid && L.op_txid[p] == u.txid;
        if (!eval_op<DMAX, true>(u, meta, ct, sv, sp, txm, p, a)) continue;
        if (scal) {
          if (t == AM_PN) pv.add(L.p0[p], 0);
          else lv.add(L.p0[p], L.p1[p]);
        } else if (!(meta & AM_META_BAD)) {
          incl |= 1ull << (p - t0);
        }
      }
    }
    pk_fold(ap, pk.K, u.allmask, a);
    int32_t status = (a.flags & FLAG_BAD) ? AM_ERR_UNEXPECTED_OPERATION : AM_OK;

    // ---- set reads: records of included ops -> born / killed groups -> survivors ----
    uint64_t galive = 0, gsrc = 0, gdst = 0;  // this lane's survivors for the wave's gather
    uint32_t ns = 0;
    if (take && setr) {
      uint64_t born = 0, killed = 0;
      for (uint64_t q = q0; q < rk1; q += 16) {
        u32x4 cv[4];
        cv[0] = rv;
#pragma unroll
        for (int j = 1; j < 4; ++j)
          cv[j] = q + 4 * j < rk1 ? *(const u32x4 *)(L.rec_g + q + 4 * j) : u32x4{~0u, ~0u, ~0u, ~0u};
        if (q + 16 < rk1) rv = *(const u32x4 *)(L.rec_g + q + 16);
#pragma unroll
        for (int j = 0; j < 4; ++j) rec_bits(cv[j], q + 4 * j, rk0, rk1, incl, sh, born, killed);
      }
      if (status == AM_OK) {
        const uint64_t alive = born & ~killed;
        ns = (uint32_t)__popcll(alive);
        const uint64_t ooff = R.value.set_off[r], ocap = R.value.set_off[r + 1] - ooff;
        if (ns > ocap) status = AM_ERR_CAPACITY;
        else galive = alive, gsrc = rk0, gdst = ooff;
      }
    }
    wave_gather(L, R, (uint32_t)__popcll(galive), galive, gsrc, gdst, lane);

    // ---- outputs ----
    if (take) {
      uint64_t v0 = 0, v1 = 0;
      uint32_t vflag = 0;
      if (t == AM_PN) {
        int64_t hi = pv.hi;
        uint64_t lo = pv.lo;
        const int64_t bv = B.base.v0 ? B.base.v0[r] : 0;
        add128(hi, lo, bv < 0 ? -1 : 0, (uint64_t)bv);
        if (status == AM_OK && hi != ((int64_t)lo < 0 ? -1 : 0)) status = AM_ERR_OVERFLOW;
        v0 = lo;
      } else if (t == AM_LWW) {
        uint64_t bts = 0, bval = 0;
        uint32_t bbin = 1;  // new() = {0, <<>>}
        if (B.base.v0) {
          bts = (uint64_t)B.base.v0[r];
          bval = B.base.v1 ? B.base.v1[r] : 0;
          bbin = B.base.vflag ? B.base.vflag[r] : 0;
        }
        const bool win = lv.has && (lv.ts > bts || (lv.ts == bts && !bbin && lv.val > bval));
        v0 = win ? lv.ts : bts;
        v1 = win ? lv.val : bval;
        vflag = win ? 0 : bbin;
      }
      write_lane(L, R, u, nd, n, r, L.key_id_base ? L.key_id_base[key] : 1, off0, off1, t, status, a, v0, v1, vflag,
                 ns);
    }
  }
}

// ================================================================ batch-clock reads
// One MinSnapshotTime for the batch, base ignore, no TxIds (the bench's and a GST read's shape).
// The work is VALU-issue-bound at this size (PMC, C4: waves issue ~90 % of the time at two waves
// per SIMD), so the kernel is built around doing little per op:
//   * persistent waves, one 64-read block at a time; block j+1's key metadata and block j+2's
//     read indices are loaded behind block j's scan loads, and block j+1 is published to the
//     other slot buffer before j's gather and output stores (a wave's loads and stores retire
//     through one in-order counter), so a block starts with nothing to wait for;
//   * publishing sorts the block's reads by type into the 64 scan positions: a phase (16
//     positions) holds one or two types, and the payload (PN sum / LWW max) and record (sets)
//     code of a type runs only in the phases that hold it (wave-uniform branches);
//   * the scan is quad-shaped: the quad at position p scans that read's first 16-op tile, lane j
//     ops [4j, 4j + 4) -- 64 contiguous bytes per packed column per quad, or with the lag view
//     (LAG) the ops' commit words and 8 bytes of u16 lags per DC, the key's lag bases published
//     with the read -- with the ops' payload or records in the same loads; the loads of QPH
//     phases are issued together;
//   * positions, inclusion bits, groups and the oldest-excluded index are 32-bit in the scan
//     (the quad takes reads of at most 16 ops and 32 groups; the thresholds S - K are computed
//     once per read by its lane and published with it); a set read ORs its included ops'
//     group masks (the gmask view: births | effective kills per op) instead of testing records;
//   * a read the quad does not take (longer logs up to 64 ops / 64 groups) is finished by its
//     own lane, and so are a quad read's escaped ops, which the quad marks (the lane evaluates
//     just those); results come back through LDS; survivors leave through one gather per wave;
//     each lane writes its read's outputs (coalesced stores).
// phases whose loads are in flight together (2 at D <= 4 measured within noise of 4)
template <int DMAX>
constexpr int qph() {
  return DMAX <= 4 ? 4 : DMAX <= 8 ? 2 : 1;
}
template <int DMAX>
struct QSlot {  // the read at a scan position, for the quad that scans it
  uint64_t off0, rk0;
  uint32_t nops, nrec, tk, ctl;  // ctl: AM_FLAG_MISSING_DC_LOGGED | never << 31
  uint32_t thr[DMAX];            // MinSnapshotTime - K per DC (pk_clamp)
  uint32_t lb[DMAX];             // the lag view: the key's lag bases (key_lag; 0 past n_dc)
};
struct QOwn {  // the lane's own read of a block (registers, from q_publish)
  uint64_t off0, K, rk0, idb, ooff;
  uint32_t nops, nrec, tk, r, ocap, pos;
};
template <int DMAX>
struct QRes {  // the quad's results for the read at position p
  uint64_t w0, w1;                 // PN 128-bit sum (hi, lo) | LWW (ts, value)
  uint32_t incl, born, killed;     // inclusion bits from off0 & ~3; groups born / killed
  uint32_t mex, count, flags;      // oldest excluded op (from off0 & ~3) or ~0; count; flags
  uint32_t escb;                   // escaped ops (from off0 & ~3): the lane evaluates just these
  uint32_t mx[DMAX];
};
constexpr uint32_t QGL = 256;  // survivor-list entries per gather round
template <int DMAX>
struct QSmem {
  QSlot<DMAX> slot[WAVE];  // by scan position; rewritten for the next block once scanned
  QRes<DMAX> res[WAVE];
  uint64_t grk0[WAVE], gdst[WAVE];  // survivor gather: group base, output base by position
  uint16_t glist[QGL];              // survivor j of the round: owner position << 6 | group
};
// tk: the read's type | taken | scanned by its quad
constexpr uint32_t QT_TAKE = 0x100u, QT_QUAD = 0x200u, QF_ESC = 0x200u, QF_HAS = 0x400u;
constexpr uint32_t QC_NEVER = 0x80000000u;

// A block read's index, key and type, and its key's metadata, as loaded: every load of a lane
// has one address and no predicate beyond validity (invalid lanes read row 0), and nothing
// loaded is combined until it is used -- so a block's metadata stays in flight behind the
// previous block's scan and the wave never waits for it early.
struct QPre {
  uint64_t key;
  uint32_t r, t, ok;  // ok: i < nsel
};
struct QMeta {
  uint64_t key, off0, off1, K, rk0, rk1, ooff, o1, idb;
  uint32_t r, t, kt, kfl, G, ok;  // ok: i < nsel and key < n_keys
};
template <bool SEL>
__device__ __forceinline__ QPre q_pre(const am_read_batch &B, const am_sel &S, uint32_t sel0, uint64_t nsel, uint64_t i) {
  QPre p;
  p.ok = i < nsel;
  const uint64_t ii = p.ok ? i : 0;
  p.r = SEL ? S.idx[sel0 + ii] : (uint32_t)ii;
  p.key = B.key[p.r];
  p.t = B.type[p.r];
  return p;
}
__device__ __forceinline__ QMeta q_meta(const am_op_log &L, const am_read_result &R, const QPre &p) {
  QMeta m;
  m.key = p.key, m.r = p.r, m.t = p.t;
  m.ok = p.ok && p.key < L.n_keys;
  const uint64_t k = m.ok ? p.key : 0;
  const uint64_t *ke = L.key_end ? L.key_end : L.key_off + 1;
  // a log without the token-group view (no set read is taken then: am_lane_accept) reads
  // dummies from key_off
  const uint64_t *rko = L.rec_key_off ? L.rec_key_off : L.key_off;
  const uint64_t *rke = L.rec_key_end ? L.rec_key_end : rko + 1;
  const uint32_t *kng = L.key_ngrp ? L.key_ngrp : (const uint32_t *)L.key_off;
  m.off0 = L.key_off[k];
  m.off1 = ke[k];
  m.kt = L.key_type[k];
  m.kfl = (L.key_flags ? L.key_flags : L.key_type)[k];  // (key_type: a dummy, unused)
  m.K = L.key_tbase[k];
  m.idb = (L.key_id_base ? L.key_id_base : L.key_off)[k];  // (key_off: a dummy, unused)
  // set fields for every read: the block's reads cover one span of each column, so the
  // lines are fetched whatever the types
  m.G = kng[k];
  m.rk0 = rko[k];
  m.rk1 = rke[k];
  const uint64_t *so = R.value.set_off ? R.value.set_off : L.key_off;  // (key_off: a dummy)
  m.ooff = so[m.r];
  m.o1 = so[m.r + 1];
  return m;
}

// A block's reads -> their scan positions in slot[]: errors get their status, reads the tier
// does not take go to `next` (one atomic per wave), the rest are placed by type (PN, LWW, AW, MV,
// then the reads their own lanes finish, then the rest).  Returns the lane's position; *any
// whether any read is taken.
template <int DMAX, bool LAG>
__device__ __forceinline__ QOwn q_publish(const am_op_log &L, const am_read_result &R, const ReadU<DMAX> &u,
                                          uint32_t nd, const QMeta &m, bool inb, uint32_t accept, am_retry next,
                                          QSlot<DMAX> *slot, uint32_t lane, bool &any) {
  const uint64_t lt = (1ull << lane) - 1ull;
  bool take = false, hand = false;
  if (inb) {
    int32_t st = AM_OK;
    if (!m.ok || m.t < AM_PN || m.t > AM_BCOUNTER) st = AM_ERR_INVALID;
    else if (m.off1 > m.off0 && (m.kt != m.t || (L.key_flags && (m.kfl & AM_KEY_MIXED_TYPES))))
      st = AM_ERR_CORRUPTED_OPS_CACHE;
    if (st == AM_OK) {
      bool ok = ((accept >> m.t) & 1u) && m.off1 - (m.off0 & ~3ull) <= LBITS;
      if (ok && (m.t == AM_AWSET || m.t == AM_MVREG)) ok = m.G != AM_NGRP_NONE && m.G <= LGRP;
      take = ok;
      hand = !ok;
    } else {
      R.status[m.r] = st;
      R.flags[m.r] = 0;
    }
  }
  const uint64_t hm = __ballot(hand);
  if (hm) {
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(next.count, (uint32_t)__popcll(hm));
    base = uniform_u32(base);
    if (hand) next.list[base + (uint32_t)__popcll(hm & lt)] = m.r;
  }
  const bool setr = m.t == AM_AWSET || m.t == AM_MVREG;
  const bool quad = take && m.off1 <= (m.off0 & ~3ull) + 16 && (!setr || (L.gmask && m.G <= AM_GMASK_MAX_GRP));
  // scan position: quad reads by type, then the lane-finished reads, then the rest
  const uint32_t cls = quad ? m.t - AM_PN : take ? 4u : 5u;
  uint32_t pos = 0;
#pragma unroll
  for (uint32_t c = 0; c < 6; ++c) {
    const uint64_t mc = __ballot(cls == c);
    if (cls == c) pos += (uint32_t)__popcll(mc & lt);
    if (cls > c) pos += (uint32_t)__popcll(mc);
  }
  QOwn o;
  o.off0 = m.off0, o.K = m.K, o.rk0 = setr ? m.rk0 : 0, o.idb = L.key_id_base ? m.idb : 1, o.ooff = m.ooff;
  o.nops = (uint32_t)(m.off1 - m.off0), o.nrec = setr ? (uint32_t)(m.rk1 - m.rk0) : 0u, o.r = m.r;
  o.ocap = setr ? (uint32_t)min(m.o1 - m.ooff, (uint64_t)0xFFFFFFFFu) : 0u;
  o.tk = take ? (m.t | QT_TAKE | (quad ? QT_QUAD : 0u)) : 0u;
  o.pos = pos;
  QSlot<DMAX> &w = slot[pos];
  w.off0 = o.off0, w.rk0 = o.rk0, w.nops = o.nops, w.nrec = o.nrec, w.tk = o.tk;
  if (quad) {  // the packed thresholds, once per read (am_wave.h pk_setup)
    PkRead<DMAX> pk;
    pk_setup(u, nd, m.K, pk);
#pragma unroll
    for (int d = 0; d < DMAX; ++d) w.thr[d] = pk.thr[d];
    w.ctl = pk.miss | (pk.never ? QC_NEVER : 0u);
    if (LAG) {
#pragma unroll
      for (int d = 0; d < DMAX; ++d) w.lb[d] = d < (int)nd ? (uint32_t)L.key_lag[m.key * nd + d] : 0u;
    }
  }
  any = __ballot(take) != 0;
  return o;
}

// The wave's survivor gather through the LDS list: the read at position p with n survivors
// (alive bits of its groups) owns entries excl .. excl + n - 1 of the wave's list; each round
// lists 256 entries (position, group), then lane j takes entries j, j + 64, ...: the group pair
// from grp[2 (rk0 + group)] into output slot gdst + entry.  All 64 lanes must be active.
template <int DMAX>
__device__ __forceinline__ void q_gather(const am_op_log &L, const am_read_result &R, QSmem<DMAX> &sm, uint64_t alive,
                                         uint64_t rk0, uint64_t ooff, uint32_t pos, uint32_t lane) {
  const uint32_t n = (uint32_t)__popcll(alive);
  const uint32_t incl = wave_incl_scan_u32(n, lane), excl = incl - n;
  const uint32_t T = lane_u32(incl, WAVE - 1);
  if (T == 0) return;
  sm.gdst[pos] = ooff - excl;
  sm.grk0[pos] = rk0;
  for (uint32_t base = 0; base < T; base += QGL) {
    uint32_t k = excl;
    for (uint64_t bits = alive; bits && k < base + QGL; bits &= bits - 1, ++k)
      if (k >= base) sm.glist[k - base] = (uint16_t)(pos << 6 | (uint32_t)__builtin_ctzll(bits));
    wave_sync();
    constexpr int K = QGL / WAVE;
    u64x2 ab[K];
    uint64_t to[K];
#pragma unroll
    for (int e = 0; e < K; ++e) {  // unpredicated loads (entry T - 1 repeated past the end)
      const uint32_t j = base + (uint32_t)e * WAVE + lane, jj = j < T ? j : T - 1;
      const uint32_t x = sm.glist[jj - base], own = x >> 6;
      to[e] = j < T ? sm.gdst[own] + j : ~0ull;
      ab[e] = *(const u64x2 *)(L.grp + 2 * (sm.grk0[own] + (x & 63u)));
    }
#pragma unroll
    for (int e = 0; e < K; ++e)
      if (to[e] != ~0ull) R.value.set_a[to[e]] = ab[e].x, R.value.set_b[to[e]] = ab[e].y;
    wave_sync();
  }
}

__device__ __forceinline__ uint64_t u64of(uint32_t lo, uint32_t hi) { return (uint64_t)hi << 32 | lo; }

// the included ops' payload of an op tile (bit k of ib: op k of the lane): PN 128-bit sum, LWW max
__device__ __forceinline__ void q_pn(uint32_t ib, u32x4 e0, u32x4 e1, PnVal &pv) {
  const uint64_t v[4] = {u64of(e0.x, e0.y), u64of(e0.z, e0.w), u64of(e1.x, e1.y), u64of(e1.z, e1.w)};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t d = ((ib >> k) & 1u) ? (int64_t)v[k] : 0;
    add128(pv.hi, pv.lo, d < 0 ? -1 : 0, (uint64_t)d);
  }
}
__device__ __forceinline__ void q_lww(uint32_t ib, u32x4 e0, u32x4 e1, u32x4 e2, u32x4 e3, LwwVal &lv) {
  const uint64_t ts[4] = {u64of(e0.x, e0.y), u64of(e0.z, e0.w), u64of(e1.x, e1.y), u64of(e1.z, e1.w)};
  const uint64_t va[4] = {u64of(e2.x, e2.y), u64of(e2.z, e2.w), u64of(e3.x, e3.y), u64of(e3.z, e3.w)};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const bool in = (ib >> k) & 1u;
    const bool gt = in && (!lv.has || ts[k] > lv.ts || (ts[k] == lv.ts && va[k] > lv.val));
    lv.ts = gt ? ts[k] : lv.ts;
    lv.val = gt ? va[k] : lv.val;
    lv.has |= in ? 1u : 0u;
  }
}
#ifndef AM_LANE_LAG
#define AM_LANE_LAG 1
#endif
template <int DMAX, bool SEL, bool LAG>
__global__ void __launch_bounds__(LBLOCK) k_lane_q(am_op_log L, am_read_batch B, am_read_result R, am_sel S,
                                                   am_retry next, uint32_t accept) {
  constexpr int NPH = qph<DMAX>();
  __shared__ QSmem<DMAX> smem[LBLOCK / WAVE];
  QSmem<DMAX> &sm = smem[threadIdx.x / WAVE];
  const uint32_t lane = threadIdx.x & (WAVE - 1), qj = lane & 3u, qq = lane >> 2;
  const uint32_t nd = L.n_dc;
  const uint64_t stride = L.snap_stride ? L.snap_stride : L.n_ops;
  const uint32_t sel0 = SEL ? uniform_u32(S.range[0]) : 0u;
  const uint64_t nsel = SEL ? (uint64_t)(uniform_u32(S.range[1]) - sel0) : B.n_reads;
  const uint64_t n = B.n_reads;
  ReadU<DMAX> u{};
  read_inputs<DMAX, false, true>(L, nd, B, 0, u);  // one clock, no bases / TxIds
  const uint64_t tx0[4] = {0, 0, 0, 0};

  const uint64_t step = (uint64_t)gridDim.x * LBLOCK;
  const uint64_t first = (uint64_t)blockIdx.x * LBLOCK + (threadIdx.x & ~(WAVE - 1));
  QSlot<DMAX> *const slot = sm.slot;
  QPre pn = q_pre<SEL>(B, S, sel0, nsel, first + step + lane);
  bool any = false;
  QOwn own = q_publish<DMAX, LAG>(L, R, u, nd, q_meta(L, R, q_pre<SEL>(B, S, sel0, nsel, first + lane)),
                             first + lane < nsel, accept, next, slot, lane, any);
  wave_sync();
  PH_DECL();
  PH_BEGIN();
  for (uint64_t b0 = first; b0 < nsel; b0 += step) {
    QMeta m;
    if (!any) {
      m = q_meta(L, R, pn);
      pn = q_pre<SEL>(B, S, sel0, nsel, b0 + 2 * step + lane);
      own = q_publish<DMAX, LAG>(L, R, u, nd, m, b0 + step + lane < nsel, accept, next, slot, lane, any);
      wave_sync();
      PH(5);
      continue;
    }
    const QOwn me = own;

    // ---- the quad scans: NPH phases' loads in flight together.  Unpredicated loads: a word a
    //      read does not need is loaded from its column's first line (one line for the whole
    //      chip, cached) and ignored, so the loads issue back to back with no branch between
    //      them and the wave's later waits count them exactly ----
#pragma unroll
    for (int pg = 0; pg < 4; pg += NPH) {
      u32x4 xv[NPH][DMAX], wv[NPH][4];
      u32x4 cv[NPH];         // LAG: the tile's lag_ct words
      uint2 lv[NPH][DMAX];   // LAG: its u16 lags, 4 per DC
#pragma unroll
      for (int h = 0; h < NPH; ++h) {
        const QSlot<DMAX> &sl = slot[16 * (pg + h) + qq];
        const uint32_t tk = sl.tk, ty = tk & 0xFFu;
        const bool qt = (tk & QT_QUAD) != 0, setr = ty == AM_AWSET || ty == AM_MVREG;
        const uint64_t o0 = sl.off0, o1 = o0 + sl.nops, g = (o0 & ~3ull) + 4 * qj;
        const bool lo = qt && g < o1;
        const uint64_t gg = lo ? g : 0;
        if constexpr (LAG) {  // 4 + 2 D bytes per op
          cv[h] = *(const u32x4 *)(L.lag_ct + gg);
#pragma unroll
          for (int d = 0; d < DMAX; ++d)
            lv[h][d] = d < (int)nd ? *(const uint2 *)(L.lag + (uint64_t)d * stride + gg) : uint2{0, 0};
        } else {
#pragma unroll
          for (int d = 0; d < DMAX; ++d)
            xv[h][d] = d < (int)nd ? *(const u32x4 *)(L.pk_vc + (uint64_t)d * stride + gg) : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {  // PN p0 | LWW p0, p1 | a set read's group masks
          const bool v = lo && (e < 2 || ty == AM_LWW);
          const uint64_t *col = setr ? L.gmask : (e < 2 ? L.p0 : L.p1);
          wv[h][e] = *(const u32x4 *)((setr && e >= 2 ? L.p0 : col) + (v ? g + 2 * (e & 1) : 0));
        }
      }
      if (pg == 0) {  // the next block's metadata, behind this block's scan loads
        m = q_meta(L, R, pn);
        pn = q_pre<SEL>(B, S, sel0, nsel, b0 + 2 * step + lane);
      }
#pragma unroll
      for (int h = 0; h < NPH; ++h) {
        const uint32_t i = 16 * (pg + h) + qq;
        const QSlot<DMAX> &sl = slot[i];
        const uint32_t tk = sl.tk, ty = tk & 0xFFu;
        const bool qt = (tk & QT_QUAD) != 0;
        // the phase's types (wave-uniform): code for a type runs only where it is present
        const bool tb = __ballot(qt && ty == AM_PN) != 0;
        const bool tl = __ballot(qt && ty == AM_LWW) != 0;
        const bool ts = __ballot(qt && (ty == AM_AWSET || ty == AM_MVREG)) != 0;
        if (!tb && !tl && !ts) continue;
        const uint32_t rel0 = (uint32_t)(sl.off0 & 3u), n0 = sl.nops, ctl = sl.ctl;
        // ---- ops [4 qj, 4 qj + 4) of the tile: is_op_in_snapshot/7 on the packed entries ----
        uint32_t ib = 0, ev = 0, esc = 0, cnt = 0, mex = 0xFFFFFFFFu;
        uint32_t mx[DMAX];
#pragma unroll
        for (int d = 0; d < DMAX; ++d) mx[d] = 0;
        if constexpr (LAG) {  // the packed entries X[d] - K = lag_ct - (lb[d] + lag[d])
          const u32x4 c = cv[h];
#pragma unroll
          for (int d = 0; d < DMAX; ++d) {
            const uint32_t b = sl.lb[d];
            const uint2 v = lv[h][d];
            xv[h][d] = u32x4{c.x - (b + (v.x & 0xFFFFu)), c.y - (b + (v.x >> 16)), c.z - (b + (v.y & 0xFFFFu)),
                             c.w - (b + (v.y >> 16))};
          }
        }
        if (qt) {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const uint32_t p = 4 * qj + (uint32_t)k;
            const bool inr = p - rel0 < n0;  // (unsigned: p < rel0 wraps)
            const uint32_t x0 = LAG ? cv[h][k] : xv[h][0][k];  // AM_PK_ESC: escaped
            const bool e = x0 == AM_PK_ESC;
            uint32_t over = 0;
#pragma unroll
            for (int d = 0; d < DMAX; ++d) over |= __builtin_elementwise_sub_sat(xv[h][d][k], sl.thr[d]);
            const bool cand = inr && !e;
            const bool in = cand && !(ctl & QC_NEVER) && over == 0;
            ib |= (uint32_t)in << k;
            ev |= (uint32_t)cand << k;
            esc |= (uint32_t)(inr && e) << k;
#pragma unroll
            for (int d = 0; d < DMAX; ++d) mx[d] = max(mx[d], in ? xv[h][d][k] : 0u);
          }
          cnt = (uint32_t)__popc(ib);
          const uint32_t ex = ev & ~ib;
          mex = ex ? 4 * qj + (uint32_t)__builtin_ctz(ex) : 0xFFFFFFFFu;
        }
        PnVal qpv;
        LwwVal qlv;
        qpv.reset();
        qlv.reset();
        if (tb && ty == AM_PN) q_pn(ib, wv[h][0], wv[h][1], qpv);
        if (tl && ty == AM_LWW) q_lww(ib, wv[h][0], wv[h][1], wv[h][2], wv[h][3], qlv);
        const uint32_t qincl = quad_or_u32(ib << (4 * qj)), qesc = quad_or_u32(esc << (4 * qj));
#pragma unroll
        for (int d = 0; d < DMAX; ++d) mx[d] = d < (int)nd ? quad_max_u32(mx[d]) : 0u;
        cnt = quad_sum_u32(cnt);
        const uint32_t fl = quad_or_u32((ev ? (ctl & AM_FLAG_MISSING_DC_LOGGED) : 0u) | (esc ? QF_ESC : 0u));
        mex = quad_min_u32(mex);
        if (tb) {
          quad_step_i128<0xB1>(qpv.hi, qpv.lo);
          quad_step_i128<0x4E>(qpv.hi, qpv.lo);
        }
        if (tl) {
          quad_step_lww<0xB1>(qlv);
          quad_step_lww<0x4E>(qlv);
        }
        // ---- set reads: the included ops' group masks -> born / killed groups ----
        uint32_t born = 0, killed = 0;
        if (ts) {
          if (ty == AM_AWSET || ty == AM_MVREG) {
            const uint32_t gw[8] = {wv[h][0].x, wv[h][0].y, wv[h][0].z, wv[h][0].w,
                                    wv[h][1].x, wv[h][1].y, wv[h][1].z, wv[h][1].w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const bool in = (ib >> k) & 1u;
              born |= in ? gw[2 * k] : 0u;
              killed |= in ? gw[2 * k + 1] : 0u;
            }
          }
          born = quad_or_u32(born);
          killed = quad_or_u32(killed);
        }
        if (qj == 0 && qt) {
          QRes<DMAX> &o = sm.res[i];
          o.w0 = ty == AM_LWW ? qlv.ts : (uint64_t)qpv.hi;
          o.w1 = ty == AM_LWW ? qlv.val : qpv.lo;
          o.incl = qincl, o.born = born, o.killed = killed, o.mex = mex, o.count = cnt, o.escb = qesc;
          o.flags = fl | (qlv.has ? QF_HAS : 0u);
#pragma unroll
          for (int d = 0; d < DMAX; ++d) o.mx[d] = mx[d];
        }
      }
    }
    PH(0);
    // the next block's reads: statuses, hand-offs, positions (its metadata has arrived by now;
    // the slots are free once scanned)
    wave_sync();
    own = q_publish<DMAX, LAG>(L, R, u, nd, m, b0 + step + lane < nsel, accept, next, slot, lane, any);
    wave_sync();
    PH(1);

    // ---- the lane's own read: its quad's results, or (a longer read) its own scan ----
    const uint32_t tk = me.tk, t = tk & 0xFFu;
    const bool tk_take = (tk & QT_TAKE) != 0;
    const bool scal = t == AM_PN || t == AM_LWW, setr = t == AM_AWSET || t == AM_MVREG;
    const uint64_t off0 = me.off0, off1 = off0 + me.nops, a0 = off0 & ~3ull, K = me.K;
    const uint64_t rk0 = me.rk0, rk1 = rk0 + me.nrec;
    AccP<DMAX> ap;
    Acc<DMAX> a;
    ap.reset();
    a.reset();
    PnVal pv;
    LwwVal lv;
    pv.reset();
    lv.reset();
    uint64_t incl = 0, born = 0, killed = 0;
    bool esc = false;
    uint32_t escb = 0;  // a quad read's escaped ops (from a0)
    if (tk & QT_QUAD) {
      const QRes<DMAX> &o = sm.res[me.pos];
      incl = o.incl, born = o.born, killed = o.killed;
      ap.min_excl = o.mex == 0xFFFFFFFFu ? NONE : a0 + o.mex;
      ap.count = o.count, ap.flags = o.flags & ~(QF_ESC | QF_HAS);
#pragma unroll
      for (int d = 0; d < DMAX; ++d) ap.mx[d] = o.mx[d];
      esc = (o.flags & QF_ESC) != 0;
      escb = o.escb;
      if (t == AM_PN) pv.hi = (int64_t)o.w0, pv.lo = o.w1;
      if (t == AM_LWW) lv.ts = o.w0, lv.val = o.w1, lv.has = (o.flags & QF_HAS) ? 1u : 0u;
    } else if (tk_take) {  // longer logs of the lane tier (up to 64 ops / 64 groups)
      PkRead<DMAX> pk;
      pk_setup(u, nd, K, pk);
      for (uint64_t g = a0; g < off1; g += 4) {
        uint32_t x[4][DMAX];
#pragma unroll
        for (int d = 0; d < DMAX; ++d) {
          const u32x4 c = d < (int)nd ? *(const u32x4 *)(L.pk_vc + (uint64_t)d * stride + g) : u32x4{0, 0, 0, 0};
          x[0][d] = c.x, x[1][d] = c.y, x[2][d] = c.z, x[3][d] = c.w;
        }
        u32x4 e0 = {0, 0, 0, 0}, e1 = e0, e2 = e0, e3 = e0;
        if (scal) e0 = *(const u32x4 *)(L.p0 + g), e1 = *(const u32x4 *)(L.p0 + g + 2);
        if (t == AM_LWW) e2 = *(const u32x4 *)(L.p1 + g), e3 = *(const u32x4 *)(L.p1 + g + 2);
        const uint32_t ib = pk_tile<DMAX, 4, false>(u, pk, x, tx0, g, off0, off1, ap, esc);
        incl |= (uint64_t)ib << (g - a0);
        if (t == AM_PN) q_pn(ib, e0, e1, pv);
        if (t == AM_LWW) q_lww(ib, e0, e1, e2, e3, lv);
      }
      for (uint64_t q = rk0 & ~3ull; setr && q < rk1; q += 4)
        rec_bits(*(const u32x4 *)(L.rec_g + q), q, rk0, rk1, incl, (uint32_t)(off0 - a0), born, killed);
    }
    if (esc) {  // rare: ops outside the packed view, from the full columns
      uint64_t ek = 0;  // included set ops among them: the records are redone with them
      auto esc_op = [&](uint64_t p) {
        uint64_t sv[DMAX], ct;
        uint32_t meta;
        esc_load<DMAX>(L, nd, stride, p, sv, ct, meta);
        if (!eval_op<DMAX, false>(u, meta, ct, sv, u.allmask, false, p, a)) return;
        if (scal) {
          if (t == AM_PN) pv.add(L.p0[p], 0);
          else lv.add(L.p0[p], L.p1[p]);
        } else if (!(meta & AM_META_BAD)) {
          ek |= 1ull << (p - a0);
        }
      };
      if (tk & QT_QUAD) {  // the quad scan marked them
        for (uint32_t m = escb; m; m &= m - 1) esc_op(a0 + (uint64_t)__builtin_ctz(m));
      } else {  // the lane's own scan of a longer log: its packed entries flag them
        for (uint64_t p = off0; p < off1; ++p)
          if (L.pk_vc[p] == AM_PK_ESC) esc_op(p);
      }
      if (setr && ek) {
        incl |= ek;
        born = 0, killed = 0;
        for (uint64_t q = rk0 & ~3ull; q < rk1; q += 4)
          rec_bits(*(const u32x4 *)(L.rec_g + q), q, rk0, rk1, incl, (uint32_t)(off0 - a0), born, killed);
      }
    }
    pk_fold(ap, K, u.allmask, a);
    int32_t status = (a.flags & FLAG_BAD) ? AM_ERR_UNEXPECTED_OPERATION : AM_OK;
    uint64_t galive = 0;
    uint32_t ns = 0;
    const uint64_t ooff = me.ooff;
    if (tk_take && setr && status == AM_OK) {
      const uint64_t alive = born & ~killed;
      ns = (uint32_t)__popcll(alive);
      if (ns > me.ocap) status = AM_ERR_CAPACITY;
      else galive = alive;
    }
    const uint64_t r = me.r, idb = me.idb;
    PH(2);
    q_gather<DMAX>(L, R, sm, galive, rk0, ooff, me.pos, lane);
    PH(3);

    if (tk_take) {
      uint64_t v0 = 0, v1 = 0;
      uint32_t vflag = 0;
      if (t == AM_PN) {
        if (status == AM_OK && pv.hi != ((int64_t)pv.lo < 0 ? -1 : 0)) status = AM_ERR_OVERFLOW;
        v0 = pv.lo;
      } else if (t == AM_LWW) {  // base new() = {0, <<>>}: any op wins
        v0 = lv.has ? lv.ts : 0;
        v1 = lv.has ? lv.val : 0;
        vflag = lv.has ? 0u : 1u;
      }
      write_lane(L, R, u, nd, n, r, idb, off0, off1, t, status, a, v0, v1, vflag, ns);
    }
    wave_sync();  // the LDS area is rewritten by the next block
    PH(4);
  }
  PH_END();
}

template <int D, bool LAG>
int launch_dl(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S, am_retry next,
              uint32_t accept, bool general) {
  static int occ_g = 0, occ_q = 0;
  int &occ = general ? occ_g : occ_q;
  if (!occ) {
    const hipError_t e = general ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_lane_g<D>, LBLOCK, 0)
                                 : hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_lane_q<D, false, LAG>, LBLOCK, 0);
    if (e != hipSuccess || occ < 1) occ = 2;
  }
  uint64_t blocks = (B->n_reads + LBLOCK - 1) / LBLOCK, cap = (uint64_t)ctx->n_cu * occ;
  if (blocks > cap) blocks = cap;
  if (blocks == 0) return AM_OK;
  if (general)
    hipLaunchKernelGGL((k_lane_g<D>), dim3((unsigned)blocks), dim3(LBLOCK), 0, ctx->stream, *L, *B, *R, S, next, accept);
  else if (S.idx)
    hipLaunchKernelGGL((k_lane_q<D, true, LAG>), dim3((unsigned)blocks), dim3(LBLOCK), 0, ctx->stream, *L, *B, *R, S,
                       next, accept);
  else
    hipLaunchKernelGGL((k_lane_q<D, false, LAG>), dim3((unsigned)blocks), dim3(LBLOCK), 0, ctx->stream, *L, *B, *R, S,
                       next, accept);
  AM_HIP(hipGetLastError());
  return AM_OK;
}
// the quad scan reads the lag view (4 + 2 D bytes per op instead of 4 D) where the store has one
template <int D>
int launch_d(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S, am_retry next,
             uint32_t accept, bool general) {
  if constexpr (D <= 16 && AM_LANE_LAG)
    if (!general && L->lag_ct && L->lag && L->key_lag) return launch_dl<D, true>(ctx, L, B, R, S, next, accept, general);
  return launch_dl<D, false>(ctx, L, B, R, S, next, accept, general);
}

int launch_g(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S, am_retry next,
             uint32_t accept, bool general) {
  const uint32_t nd = L->n_dc;
  if (nd <= 1) return launch_d<1>(ctx, L, B, R, S, next, accept, general);
  if (nd <= 2) return launch_d<2>(ctx, L, B, R, S, next, accept, general);
  if (nd <= 3) return launch_d<3>(ctx, L, B, R, S, next, accept, general);
  if (nd <= 4) return launch_d<4>(ctx, L, B, R, S, next, accept, general);
  if (nd <= 8) return launch_d<8>(ctx, L, B, R, S, next, accept, general);
  if (nd <= 16) return launch_d<16>(ctx, L, B, R, S, next, accept, general);
  return launch_d<32>(ctx, L, B, R, S, next, accept, general);
}

}  // namespace

#ifdef AMK_PHASE_PROF
// experiments only: read and clear the batch-clock lane kernel's phase cycle sums
extern "C" int am_debug_lane_phase_cycles(uint64_t *out) {
  unsigned long long h[8] = {0};
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(amk_grp::amk_phase_cycles), sizeof(h)) != hipSuccess) return AM_ERR_HIP;
  for (int i = 0; i < 8; ++i) out[i] = h[i];
  const unsigned long long z[8] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(amk_grp::amk_phase_cycles), z, sizeof(z)) == hipSuccess ? AM_OK : AM_ERR_HIP;
}
#endif

uint32_t am_lane_accept(const am_op_log *L, const am_read_result *R, uint32_t types) {
  if (!am_log_packed(L)) return 0;
  uint32_t acc = 0;
  if ((types & (1u << AM_PN)) && R->value.v0) acc |= 1u << AM_PN;
  if ((types & (1u << AM_LWW)) && R->value.v0 && R->value.v1 && R->value.vflag) acc |= 1u << AM_LWW;
  if ((types & (1u << AM_AWSET)) && am_group_applies(L, R, AM_AWSET)) acc |= 1u << AM_AWSET;
  if ((types & (1u << AM_MVREG)) && am_group_applies(L, R, AM_MVREG)) acc |= 1u << AM_MVREG;
  return acc;
}

int am_launch_lanes(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S,
                    am_retry next, uint32_t accept) {
  return launch_g(ctx, L, B, R, S, next, accept, am_batch_general(L, B));
}
