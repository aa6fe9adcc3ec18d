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

// experiment switch (phase costs; default off): bit 0 skips the PN / LWW payload loads, bit 1
// the set records, bit 2 the survivor gathers, bit 3 every output but the status
#ifndef AMK_LANE_SKIP
#define AMK_LANE_SKIP 0
#endif

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

template <int DMAX, int OPL>
struct LTile {
  uint32_t x[OPL][DMAX];
  uint64_t tx[OPL];
  uint64_t v0[OPL], v1[OPL];
};

#ifndef AMK_LANE_PH_UNROLL
#define AMK_LANE_PH_UNROLL 1  // quad-scan phases unrolled (experiment switch)
#endif
// waves per SIMD the register allocation must allow (experiment switch; 1 = the compiler's choice)
#ifndef AMK_LANE_MINW
#define AMK_LANE_MINW 1
#endif

template <int DMAX, bool GENERAL>
__global__ void __launch_bounds__(LBLOCK, AMK_LANE_MINW) k_lane(am_op_log L, am_read_batch B, am_read_result R, am_sel S,
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
  if (!GENERAL) read_inputs<DMAX, false, true>(L, nd, B, 0, u);  // one clock, no bases / TxIds

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
    if (GENERAL && take) read_inputs<DMAX, true, false>(L, nd, B, r, u);
    PkRead<DMAX> pk;
    pk_setup(u, nd, take ? L.key_tbase[key] : 0, pk);
    const uint64_t t0 = off0 & ~(uint64_t)(OPL - 1);
    const uint32_t sh = (uint32_t)(off0 - t0);
    // the first record vector of a set read is in flight with the ops
    const uint64_t q0 = rk0 & ~3ull;
    u32x4 rv = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    if (!(AMK_LANE_SKIP & 2) && take && setr && rk1 > rk0) rv = *(const u32x4 *)(L.rec_g + q0);

    auto load = [&](LTile<DMAX, OPL> &T, uint64_t g) {
#pragma unroll
      for (int d = 0; d < DMAX; ++d) {
        uint32_t q[OPL] = {};
        if (d < (int)nd) ld_n32<OPL>(L.pk_vc + (uint64_t)d * stride + g, q);
#pragma unroll
        for (int k = 0; k < OPL; ++k) T.x[k][d] = q[k];
      }
#pragma unroll
      for (int k = 0; k < OPL; ++k) T.tx[k] = 0, T.v0[k] = 0, T.v1[k] = 0;
      if (GENERAL && u.has_txid) ld_n64<OPL>(L.op_txid + g, T.tx);
      if (!(AMK_LANE_SKIP & 1) && scal) ld_n64<OPL>(L.p0 + g, T.v0);
      if (!(AMK_LANE_SKIP & 1) && t == AM_LWW) ld_n64<OPL>(L.p1 + g, T.v1);
    };
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
    if constexpr (!GENERAL) {
      // The scan in QUAD shape: the wave's 64 reads in 4 phases of 16; in phase ph quad q
      // (lanes 4q..4q+3) scans read 16 ph + q, lane j of the quad holding ops [4j, 4j+4) of each
      // 16-op tile, so each packed column / payload load is 64 / 128 contiguous bytes per quad
      // (one lane per read reading its own 64-byte segments: 5.0 TB/s on C4's columns, this
      // shape 6.3, scripts/bw_probe_c4.hip).  The quad's partials are combined by DPP and handed
      // to the read's own lane (ds_bpermute), which carries on as before.
      const uint32_t qj = lane & 3u;
      const uint32_t tk = take ? (t | 0x100u) : 0u;
#pragma unroll AMK_LANE_PH_UNROLL
      for (uint32_t ph = 0; ph < 4; ++ph) {
        const uint32_t src = 16u * ph + (lane >> 2);
        const uint32_t qt = shfl_u32(tk, src);
        const uint64_t qo0 = shfl_u64(off0, src), qo1 = shfl_u64(off1, src), qK = shfl_u64(pk.K, src);
        const bool qtake = (qt >> 8) & 1u;
        const uint32_t qty = qt & 0xFFu;
        PkRead<DMAX> qpk;
        pk_setup(u, nd, qK, qpk);
        const uint64_t qt0 = qo0 & ~(uint64_t)(OPL - 1);  // the owner's inclusion-bit window
        AccP<DMAX> qap;
        qap.reset();
        PnVal qpv;
        LwwVal qlv;
        qpv.reset();
        qlv.reset();
        bool qesc = false;
        uint64_t qincl = 0;
        for (uint64_t g = (qo0 & ~3ull) + 4 * qj; qtake && g < qo1; g += 16) {
          uint32_t x[4][DMAX];
#pragma unroll
          for (int d = 0; d < DMAX; ++d) {
            u32x4 q = {0, 0, 0, 0};
            if (d < (int)nd) q = *(const u32x4 *)(L.pk_vc + (uint64_t)d * stride + g);
            x[0][d] = q.x, x[1][d] = q.y, x[2][d] = q.z, x[3][d] = q.w;
          }
          u64x2 a0 = {0, 0}, a1 = {0, 0}, c0 = {0, 0}, c1 = {0, 0};
          if (!(AMK_LANE_SKIP & 1) && (qty == AM_PN || qty == AM_LWW))
            a0 = *(const u64x2 *)(L.p0 + g), a1 = *(const u64x2 *)(L.p0 + g + 2);
          if (!(AMK_LANE_SKIP & 1) && qty == AM_LWW) c0 = *(const u64x2 *)(L.p1 + g), c1 = *(const u64x2 *)(L.p1 + g + 2);
          const uint64_t tx[4] = {0, 0, 0, 0};
          const uint32_t ib = pk_tile<DMAX, 4, false>(u, qpk, x, tx, g, qo0, qo1, qap, qesc);
          qincl |= (uint64_t)ib << (g - qt0);
          const uint64_t pv0[4] = {a0.x, a0.y, a1.x, a1.y}, pv1[4] = {c0.x, c0.y, c1.x, c1.y};
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if ((ib >> k) & 1u) {
              if (qty == AM_PN) qpv.add(pv0[k], 0);
              else if (qty == AM_LWW) qlv.add(pv0[k], pv1[k]);
            }
        }
        qincl = quad_or_u64(qincl);
#pragma unroll
        for (int d = 0; d < DMAX; ++d) qap.mx[d] = quad_max_u32(qap.mx[d]);
        qap.count = quad_sum_u32(qap.count);
        qap.flags = quad_or_u32(qap.flags | (qesc ? 0x200u : 0u));
        qap.min_excl = quad_min_u64(qap.min_excl);
        quad_step_i128<0xB1>(qpv.hi, qpv.lo);
        quad_step_i128<0x4E>(qpv.hi, qpv.lo);
        quad_step_lww<0xB1>(qlv);
        quad_step_lww<0x4E>(qlv);
        // PN and LWW reads are exclusive: one payload pair travels
        const uint64_t w0 = qty == AM_LWW ? qlv.ts : (uint64_t)qpv.hi, w1 = qty == AM_LWW ? qlv.val : qpv.lo;
        const uint32_t fl = qap.flags | (qlv.has ? 0x400u : 0u);
        // the read's own lane (16 ph + q) takes its quad's values from quad lane 0
        const uint32_t from = (lane >> 4) == ph ? 4u * (lane & 15u) : lane;
        const uint64_t r_incl = shfl_u64(qincl, from), r_me = shfl_u64(qap.min_excl, from);
        const uint64_t r_w0 = shfl_u64(w0, from), r_w1 = shfl_u64(w1, from);
        const uint32_t r_cnt = shfl_u32(qap.count, from), r_fl = shfl_u32(fl, from);
        uint32_t r_mx[DMAX];
#pragma unroll
        for (int d = 0; d < DMAX; ++d) r_mx[d] = d < (int)nd ? shfl_u32(qap.mx[d], from) : 0u;
        if ((lane >> 4) == ph) {
          incl = r_incl;
#pragma unroll
          for (int d = 0; d < DMAX; ++d) ap.mx[d] = r_mx[d];
          ap.count = r_cnt;
          ap.flags = r_fl & ~0x600u;
          ap.min_excl = r_me;
          esc = (r_fl & 0x200u) != 0;
          if (t == AM_PN) pv.hi = (int64_t)r_w0, pv.lo = r_w1;
          if (t == AM_LWW) lv.ts = r_w0, lv.val = r_w1, lv.has = (r_fl & 0x400u) ? 1u : 0u;
        }
      }
    } else {
      LTile<DMAX, OPL> cur;
      for (uint64_t g = t0; take && g < off1; g += OPL) {
        load(cur, g);
        const uint32_t ib = pk_tile<DMAX, OPL, GENERAL>(u, pk, cur.x, cur.tx, g, off0, off1, ap, esc);
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
    }
    if (esc) {  // rare: ops outside the packed view, from the full columns
      for (uint64_t p = off0; p < off1; ++p) {
        if (L.pk_vc[p] != AM_PK_ESC) continue;
        uint64_t sv[DMAX];
#pragma unroll
        for (int d = 0; d < DMAX; ++d) sv[d] = d < (int)nd ? L.snap_vc[(uint64_t)d * stride + p] : 0;
        const uint32_t meta = L.op_meta[p];
        const uint32_t sp = (GENERAL && L.snap_pres) ? L.snap_pres[p] : u.allmask;
        const bool txm = GENERAL && u.has_txid && L.op_txid[p] == u.txid;
        if (!eval_op<DMAX, GENERAL>(u, meta, L.commit_time[p], sv, sp, txm, p, a)) continue;
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
    uint32_t ns = 0;
    uint64_t galive = 0, gsrc = 0, gdst = 0;  // this lane's survivors for the wave's gather
    if (take && setr) {
      uint64_t born = 0, killed = 0;
      // 16 records per step: the first vector was prefetched with the ops, the other three
      // are loaded together (an MV read of 16 ops has 31 records: two steps, not eight)
      for (uint64_t q = q0; !(AMK_LANE_SKIP & 2) && q < rk1; q += 16) {
        u32x4 cv[4];
        cv[0] = rv;
#pragma unroll
        for (int j = 1; j < 4; ++j)
          cv[j] = q + 4 * j < rk1 ? *(const u32x4 *)(L.rec_g + q + 4 * j) : u32x4{~0u, ~0u, ~0u, ~0u};
        if (q + 16 < rk1) rv = *(const u32x4 *)(L.rec_g + q + 16);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t xs[4] = {cv[j].x, cv[j].y, cv[j].z, cv[j].w};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const uint64_t qq = q + 4 * j + k;
            const uint32_t x = xs[k];
            if (qq < rk0 || qq >= rk1 || x == 0xFFFFFFFFu) continue;
            if (!((incl >> (AM_REC_OP(x) + sh)) & 1ull)) continue;
            const uint64_t bit = 1ull << AM_REC_GRP(x);
            if (x & AM_REC_KILL) killed |= bit;
            else born |= bit;
          }
        }
      }
      if (status == AM_OK) {
        const uint64_t alive = born & ~killed;
        ns = (uint32_t)__popcll(alive);
        const uint64_t ooff = R.value.set_off[r], ocap = R.value.set_off[r + 1] - ooff;
        if (ns > ocap) {
          status = AM_ERR_CAPACITY;
        } else if (!(AMK_LANE_SKIP & 4)) {
          galive = alive, gsrc = rk0, gdst = ooff;
        }
      }
    }
    // survivors of every set read of the wave in one gather: the wave's concatenated survivor
    // list (read order, group order within a read) is split over all 64 lanes, so a wave issues
    // up to 256 independent 16-byte group loads at once and writes each read's pairs with
    // adjacent lanes (one lane per read looping over its survivors serialized a memory
    // latency per four survivors)
    wave_gather(L, R, (uint32_t)__popcll(galive), galive, gsrc, gdst, lane);

    // ---- outputs ----
    if (take) {
      uint64_t v0 = 0, v1 = 0;
      uint32_t vflag = 0;
      if (t == AM_PN) {
        int64_t hi = pv.hi;
        uint64_t lo = pv.lo;
        const int64_t bv = (GENERAL && B.base.v0) ? B.base.v0[r] : 0;
        add128(hi, lo, bv < 0 ? -1 : 0, (uint64_t)bv);
        if (status == AM_OK && hi != ((int64_t)lo < 0 ? -1 : 0)) status = AM_ERR_OVERFLOW;
        v0 = lo;
      } else if (t == AM_LWW) {
        uint64_t bts = 0, bval = 0;
        uint32_t bbin = 1;  // new() = {0, <<>>}
        if (GENERAL && B.base.v0) {
          bts = (uint64_t)B.base.v0[r];
          bval = B.base.v1 ? B.base.v1[r] : 0;
          bbin = B.base.vflag ? B.base.vflag[r] : 0;
        }
        const bool win = lv.has && (lv.ts > bts || (lv.ts == bts && !bbin && lv.val > bval));
        v0 = win ? lv.ts : bts;
        v1 = win ? lv.val : bval;
        vflag = win ? 0 : bbin;
      }
      R.status[r] = status;
      if (AMK_LANE_SKIP & 8) continue;
      R.flags[r] = (uint8_t)(a.flags & 0xFFu);
      if (status == AM_OK) {
        R.new_last_op[r] = new_last_op(L, key, off0, off1, a.min_excl);
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
        if (scal) R.value.v0[r] = (int64_t)v0;
        if (t == AM_LWW) {
          R.value.v1[r] = v1;
          R.value.vflag[r] = (uint8_t)vflag;
        }
        if (setr) R.value.set_len[r] = ns;
      }
    }
  }
}

template <int D, bool GENERAL>
int launch_d(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S, am_retry next,
             uint32_t accept) {
  static int occ = 0;
  if (!occ) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_lane<D, GENERAL>, LBLOCK, 0) != hipSuccess || occ < 1)
      occ = 2;
  }
  uint64_t blocks = (B->n_reads + LBLOCK - 1) / LBLOCK, cap = (uint64_t)ctx->n_cu * occ;
  if (blocks > cap) blocks = cap;
  if (blocks == 0) return AM_OK;
  hipLaunchKernelGGL((k_lane<D, GENERAL>), dim3((unsigned)blocks), dim3(LBLOCK), 0, ctx->stream, *L, *B, *R, S, next,
                     accept);
  AM_HIP(hipGetLastError());
  return AM_OK;
}

template <bool GENERAL>
int launch_g(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S, am_retry next,
             uint32_t accept) {
  const uint32_t nd = L->n_dc;
  if (nd <= 1) return launch_d<1, GENERAL>(ctx, L, B, R, S, next, accept);
  if (nd <= 2) return launch_d<2, GENERAL>(ctx, L, B, R, S, next, accept);
  if (nd <= 3) return launch_d<3, GENERAL>(ctx, L, B, R, S, next, accept);
  if (nd <= 4) return launch_d<4, GENERAL>(ctx, L, B, R, S, next, accept);
  if (nd <= 8) return launch_d<8, GENERAL>(ctx, L, B, R, S, next, accept);
  if (nd <= 16) return launch_d<16, GENERAL>(ctx, L, B, R, S, next, accept);
  return launch_d<32, GENERAL>(ctx, L, B, R, S, next, accept);
}

}  // namespace

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
  return am_batch_general(L, B) ? launch_g<true>(ctx, L, B, R, S, next, accept)
                                : launch_g<false>(ctx, L, B, R, S, next, accept);
}
