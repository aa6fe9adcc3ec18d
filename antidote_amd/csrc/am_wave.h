// am_wave.h -- wave64 building blocks shared by the materialize kernels:
// DPP row reductions, wave-uniform helpers, and the per-op inclusion test of
// clocksi_materializer:is_op_in_snapshot/7.
#pragma once
#include "am_internal.h"

namespace amk {

constexpr int WAVE = 64;
constexpr uint64_t NONE = ~0ull;

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t uniform_u32(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uniform_u64(uint64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t lane_u32(uint32_t v, uint32_t l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint64_t lane_u64(uint64_t v, uint32_t l) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}

// ---- DPP: butterflies inside a 16-lane row (quad_perm 1032 / 2301, row_ror 4 / 8) ----
// Every lane of a row ends with the row's reduction; the four rows are then
// combined from lanes 0/16/32/48 with v_readlane (result is wave-uniform).
// Requires all 64 lanes active.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ uint64_t dpp64(uint64_t v) {
  return ((uint64_t)dpp32<CTRL>((uint32_t)(v >> 32)) << 32) | dpp32<CTRL>((uint32_t)v);
}
#define AMK_ROW_STEPS(STEP) STEP(0xB1) STEP(0x4E) STEP(0x124) STEP(0x128)

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#define S_(C) v += dpp32<C>(v);
  AMK_ROW_STEPS(S_)
#undef S_
  return lane_u32(v, 0) + lane_u32(v, 16) + lane_u32(v, 32) + lane_u32(v, 48);
}
__device__ __forceinline__ uint32_t wave_or_u32(uint32_t v) {
#define S_(C) v |= dpp32<C>(v);
  AMK_ROW_STEPS(S_)
#undef S_
  return lane_u32(v, 0) | lane_u32(v, 16) | lane_u32(v, 32) | lane_u32(v, 48);
}
__device__ __forceinline__ uint64_t umax64(uint64_t a, uint64_t b) { return a > b ? a : b; }
__device__ __forceinline__ uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#define S_(C) v = umax64(v, dpp64<C>(v));
  AMK_ROW_STEPS(S_)
#undef S_
  return umax64(umax64(lane_u64(v, 0), lane_u64(v, 16)), umax64(lane_u64(v, 32), lane_u64(v, 48)));
}
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#define S_(C) v = umin64(v, dpp64<C>(v));
  AMK_ROW_STEPS(S_)
#undef S_
  return umin64(umin64(lane_u64(v, 0), lane_u64(v, 16)), umin64(lane_u64(v, 32), lane_u64(v, 48)));
}
// The same reductions with the result left in every lane's VGPRs (no readlane to scalar
// registers): for kernels whose scalar register file is already full.
__device__ __forceinline__ uint64_t xor_u64(uint64_t v, int m) {
  const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m, WAVE);
  const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m, WAVE);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t wave_sum_u32_v(uint32_t v) {
#define S_(C) v += dpp32<C>(v);
  AMK_ROW_STEPS(S_)
#undef S_
  v += (uint32_t)__shfl_xor((int)v, 16, WAVE);
  return v + (uint32_t)__shfl_xor((int)v, 32, WAVE);
}
__device__ __forceinline__ uint32_t wave_or_u32_v(uint32_t v) {
#define S_(C) v |= dpp32<C>(v);
  AMK_ROW_STEPS(S_)
#undef S_
  v |= (uint32_t)__shfl_xor((int)v, 16, WAVE);
  return v | (uint32_t)__shfl_xor((int)v, 32, WAVE);
}
__device__ __forceinline__ uint32_t wave_max_u32_v(uint32_t v) {
#define S_(C) v = max(v, dpp32<C>(v));
  AMK_ROW_STEPS(S_)
#undef S_
  v = max(v, (uint32_t)__shfl_xor((int)v, 16, WAVE));
  return max(v, (uint32_t)__shfl_xor((int)v, 32, WAVE));
}
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v, uint32_t lane) {
#pragma unroll
  for (int o = 1; o < WAVE; o <<= 1) {
    const uint32_t t = (uint32_t)__shfl_up((int)v, (unsigned)o, WAVE);
    if (lane >= (uint32_t)o) v += t;
  }
  return v;
}
__device__ __forceinline__ uint64_t wave_max_u64_v(uint64_t v) {
#define S_(C) v = umax64(v, dpp64<C>(v));
  AMK_ROW_STEPS(S_)
#undef S_
  v = umax64(v, xor_u64(v, 16));
  return umax64(v, xor_u64(v, 32));
}
__device__ __forceinline__ uint64_t wave_min_u64_v(uint64_t v) {
#define S_(C) v = umin64(v, dpp64<C>(v));
  AMK_ROW_STEPS(S_)
#undef S_
  v = umin64(v, xor_u64(v, 16));
  return umin64(v, xor_u64(v, 32));
}
// exact 128-bit sum of per-lane (hi, lo) pairs
__device__ __forceinline__ void add128(int64_t &hi, uint64_t &lo, int64_t whi, uint64_t wlo) {
  const uint64_t s = lo + wlo;
  hi = hi + whi + (s < lo ? 1 : 0);
  lo = s;
}
__device__ __forceinline__ void wave_sum_i128(int64_t &hi, uint64_t &lo) {
#define S_(C)                                                     \
  {                                                               \
    const uint64_t wlo = dpp64<C>(lo);                            \
    const int64_t whi = (int64_t)dpp64<C>((uint64_t)hi);          \
    add128(hi, lo, whi, wlo);                                     \
  }
  AMK_ROW_STEPS(S_)
#undef S_
  int64_t h = (int64_t)lane_u64((uint64_t)hi, 0);
  uint64_t l = lane_u64(lo, 0);
#pragma unroll
  for (int r = 16; r < 64; r += 16) add128(h, l, (int64_t)lane_u64((uint64_t)hi, r), lane_u64(lo, r));
  hi = h;
  lo = l;
}

// ---- 16-lane row helpers (the row tier, am_rows.hip, and the group tier's row kernel) ----
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// ---- 16-lane row all-reductions: every lane of a row ends with the row's value.
// Full EXEC required (DPP reads inactive lanes as 0).
__device__ __forceinline__ uint32_t row_sum_u32(uint32_t v) {
#define S_(C) v += dpp32<C>(v);
  AMK_ROW_STEPS(S_)
#undef S_
  return v;
}
__device__ __forceinline__ uint32_t row_or_u32(uint32_t v) {
#define S_(C) v |= dpp32<C>(v);
  AMK_ROW_STEPS(S_)
#undef S_
  return v;
}
__device__ __forceinline__ uint64_t row_max_u64(uint64_t v) {
#define S_(C) v = umax64(v, dpp64<C>(v));
  AMK_ROW_STEPS(S_)
#undef S_
  return v;
}
__device__ __forceinline__ uint64_t row_min_u64(uint64_t v) {
#define S_(C) v = umin64(v, dpp64<C>(v));
  AMK_ROW_STEPS(S_)
#undef S_
  return v;
}
__device__ __forceinline__ void row_sum_i128(int64_t &hi, uint64_t &lo) {
#define S_(C)                                            \
  {                                                      \
    const uint64_t wlo = dpp64<C>(lo);                   \
    const int64_t whi = (int64_t)dpp64<C>((uint64_t)hi); \
    add128(hi, lo, whi, wlo);                            \
  }
  AMK_ROW_STEPS(S_)
#undef S_
}
__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, uint32_t src) {
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, (int)src, WAVE);
  const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), (int)src, WAVE);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t shfl_u32(uint32_t v, uint32_t src) {
  return (uint32_t)__shfl((int)v, (int)src, WAVE);
}

// ---- per-read uniform inputs and per-lane accumulators ----
template <int DMAX>
struct ReadU {
  uint64_t S[DMAX];   // MinSnapshotTime (absent lanes 0)
  uint64_t C0[DMAX];  // base snapshot_time (absent lanes 0)
  uint32_t spres, cpres, allmask;
  bool base_ignore, has_txid;
  uint64_t txid;
};

template <int DMAX>
struct Acc {
  uint64_t mx[DMAX];
  uint32_t pres, count, flags;
  uint64_t min_excl;
  __device__ void reset() {
#pragma unroll
    for (int d = 0; d < DMAX; ++d) mx[d] = 0;
    pres = count = flags = 0;
    min_excl = NONE;
  }
};

constexpr uint32_t FLAG_BAD = 0x100u;

// One op of is_op_in_snapshot/7 (src/clocksi_materializer.erl:216-268) + the
// union-max of materialize_intern_perform (:173-197).  Returns "included".
template <int DMAX, bool GENERAL>
__device__ __forceinline__ bool eval_op(const ReadU<DMAX> &u, uint32_t meta, uint64_t ct, const uint64_t (&snap)[DMAX],
                                        uint32_t spres_op, bool txmatch, uint64_t pos, Acc<DMAX> &a) {
  const uint32_t dc = meta & 31u;
  const uint32_t xpres = GENERAL ? ((spres_op | (1u << dc)) & u.allmask) : u.allmask;
  uint64_t X[DMAX];
#pragma unroll
  for (int d = 0; d < DMAX; ++d) X[d] = ((uint32_t)d == dc) ? ct : (((xpres >> d) & 1u) ? snap[d] : 0);
  if (GENERAL) {
    bool cand = u.base_ignore | txmatch;
    if (!cand) {  // belongs_to_snapshot_op: not vectorclock:le(X, base)
      bool le = true;
#pragma unroll
      for (int d = 0; d < DMAX; ++d) le &= X[d] <= u.C0[d];
      cand = !le;
    }
    if (!cand) return false;
  }
  bool incl = true;
#pragma unroll
  for (int d = 0; d < DMAX; ++d) {
    if ((xpres >> d) & 1u) {
      if ((u.spres >> d) & 1u) {
        incl &= X[d] <= u.S[d];
      } else {  // logger:error("Could not find DC in SS"); the op is excluded
        incl = false;
        a.flags |= AM_FLAG_MISSING_DC_LOGGED;
      }
    }
  }
  if (incl) {
#pragma unroll
    for (int d = 0; d < DMAX; ++d) a.mx[d] = X[d] > a.mx[d] ? X[d] : a.mx[d];
    a.pres |= xpres;
    a.count += 1;
    if (meta & AM_META_BAD) a.flags |= FLAG_BAD;
  } else {
    a.min_excl = pos < a.min_excl ? pos : a.min_excl;
  }
  return incl;
}

// ---- the same test on the packed view (am_pack.hip): the op's commit vector X as u32
// entries x[d] = X[d] - K relative to the key's time base K (every DC present).  Per read the
// clocks become u32 thresholds: X <= S iff S >= K and x <= min(S - K, 2^32 - 2), so the test
// is one compare per DC and LastOpCt one u32 max per DC.
template <int DMAX>
struct PkRead {
  uint64_t K;
  uint32_t thr[DMAX];   // MinSnapshotTime
  uint32_t cthr[DMAX];  // base snapshot_time (belongs_to_snapshot_op)
  uint32_t miss;        // AM_FLAG_MISSING_DC_LOGGED: a DC of the ops is not in the clock
  bool never;           // no op passes: a DC missing from the clock or below K
  bool cnever;          // le(X, base) fails for every op: a base entry below K
};
__device__ __forceinline__ uint32_t pk_clamp(uint64_t s, uint64_t K) {
  return s < K ? 0u : (s - K >= (uint64_t)AM_PK_ESC ? AM_PK_ESC - 1u : (uint32_t)(s - K));
}
// nd: DCs of the log; thresholds of pad lanes d >= nd pass (their entries are loaded as 0)
template <int DMAX>
__device__ __forceinline__ void pk_setup(const ReadU<DMAX> &u, uint32_t nd, uint64_t K, PkRead<DMAX> &t) {
  t.K = K;
  t.miss = (u.allmask & ~u.spres) ? AM_FLAG_MISSING_DC_LOGGED : 0u;
  t.never = t.miss != 0;
  t.cnever = false;
#pragma unroll
  for (int d = 0; d < DMAX; ++d) {
    if (d >= (int)nd) {
      t.thr[d] = AM_PK_ESC, t.cthr[d] = AM_PK_ESC;
      continue;
    }
    t.never |= u.S[d] < K;
    t.cnever |= u.C0[d] < K;
    t.thr[d] = pk_clamp(u.S[d], K);
    t.cthr[d] = pk_clamp(u.C0[d], K);
  }
}
template <int DMAX>
struct AccP {
  uint32_t mx[DMAX];
  uint32_t count, flags;
  uint64_t min_excl;
  __device__ void reset() {
#pragma unroll
    for (int d = 0; d < DMAX; ++d) mx[d] = 0;
    count = flags = 0;
    min_excl = NONE;
  }
};
// An escaped op's full-width inputs (is_op_in_snapshot/7): its escape row when the log has one
// (am_op_log.esc_rows, index + 1 in the op's DC-1 packed entry; null otherwise -- and for an op
// that is not escaped, whose DC-1 entry is a time: full-view callers may ask for any op)
__device__ __forceinline__ const uint64_t *esc_row(const am_op_log &L, uint64_t stride, uint64_t p) {
  if (!L.esc_rows || L.pk_vc[p] != AM_PK_ESC) return nullptr;
  const uint32_t ri = L.pk_vc[stride + p];
  return ri ? L.esc_rows + (uint64_t)(ri - 1) * (2 + L.n_dc) : nullptr;
}
// commit time, meta byte and snapshot entries of escaped op p: one row, or the op columns
template <int DMAX>
__device__ __forceinline__ void esc_load(const am_op_log &L, uint32_t nd, uint64_t stride, uint64_t p,
                                         uint64_t (&sv)[DMAX], uint64_t &ct, uint32_t &meta) {
  if (const uint64_t *w = esc_row(L, stride, p)) {
    ct = w[0], meta = (uint32_t)w[1];
#pragma unroll
    for (int d = 0; d < DMAX; ++d) sv[d] = d < (int)nd ? w[2 + d] : 0;
    return;
  }
  ct = L.commit_time[p], meta = L.op_meta[p];
#pragma unroll
  for (int d = 0; d < DMAX; ++d) sv[d] = d < (int)nd ? L.snap_vc[(uint64_t)d * stride + p] : 0;
}

// x[0] == AM_PK_ESC ops are the caller's (full columns)
template <int DMAX, bool GENERAL>
__device__ __forceinline__ bool pk_eval(const PkRead<DMAX> &t, const ReadU<DMAX> &u, const uint32_t (&x)[DMAX],
                                        bool txmatch, uint64_t pos, AccP<DMAX> &a) {
  if (GENERAL) {
    bool cand = u.base_ignore | txmatch;
    if (!cand) {  // belongs_to_snapshot_op: not vectorclock:le(X, base)
      bool le = !t.cnever;
#pragma unroll
      for (int d = 0; d < DMAX; ++d) le &= x[d] <= t.cthr[d];
      cand = !le;
    }
    if (!cand) return false;
  }
  a.flags |= t.miss;
  bool incl = !t.never;
#pragma unroll
  for (int d = 0; d < DMAX; ++d) incl &= x[d] <= t.thr[d];
  if (incl) {
#pragma unroll
    for (int d = 0; d < DMAX; ++d) a.mx[d] = max(a.mx[d], x[d]);
    a.count += 1;
  } else {
    a.min_excl = pos < a.min_excl ? pos : a.min_excl;
  }
  return incl;
}
// folds a lane's packed partials into its full-width accumulator (every DC present)
template <int DMAX>
__device__ __forceinline__ void pk_fold(const AccP<DMAX> &p, uint64_t K, uint32_t allmask, Acc<DMAX> &a) {
  if (p.count) {
#pragma unroll
    for (int d = 0; d < DMAX; ++d) a.mx[d] = umax64(a.mx[d], K + p.mx[d]);
    a.pres |= allmask;
  }
  a.count += p.count;
  a.flags |= p.flags;
  a.min_excl = umin64(a.min_excl, p.min_excl);
}

// the OPL packed-view ops [g, g + OPL) of a read's [off0, off1), entries x already loaded:
// inclusion bits (is_op_in_snapshot/7), partials in ap.  Branch-free: x - thr saturates to 0
// iff x <= thr, so one OR per op tests every DC; LastOpCt takes the included ops' entries
// through max chains.  An escaped op (x[k][0] == AM_PK_ESC) only sets esc.
template <int DMAX, int OPL, bool GENERAL>
__device__ __forceinline__ uint32_t pk_tile(const ReadU<DMAX> &u, const PkRead<DMAX> &pk, const uint32_t (&x)[OPL][DMAX],
                                            const uint64_t (&tx)[OPL], uint64_t g, uint64_t off0, uint64_t off1,
                                            AccP<DMAX> &ap, bool &esc) {
  uint32_t ib = 0, ev = 0;  // ev: evaluated (in range, in the packed view, a candidate)
#pragma unroll
  for (int k = 0; k < OPL; ++k) {
    const uint64_t p = g + k;
    const bool inr = p >= off0 && p < off1;
    const bool e = x[k][0] == AM_PK_ESC;
    esc |= inr && e;
    uint32_t over = 0;
#pragma unroll
    for (int d = 0; d < DMAX; ++d) over |= __builtin_elementwise_sub_sat(x[k][d], pk.thr[d]);
    bool cand = inr && !e;
    if (GENERAL) {  // belongs_to_snapshot_op: not vectorclock:le(X, base)
      uint32_t cov = 0;
#pragma unroll
      for (int d = 0; d < DMAX; ++d) cov |= __builtin_elementwise_sub_sat(x[k][d], pk.cthr[d]);
      const bool le = !pk.cnever && cov == 0;
      cand = cand && (u.base_ignore || (u.has_txid && tx[k] == u.txid) || !le);
    }
    ib |= (uint32_t)(cand && !pk.never && over == 0) << k;
    ev |= (uint32_t)cand << k;
  }
#pragma unroll
  for (int d = 0; d < DMAX; ++d) {
    uint32_t m = ap.mx[d];
#pragma unroll
    for (int k = 0; k < OPL; ++k) m = max(m, ((ib >> k) & 1u) ? x[k][d] : 0u);
    ap.mx[d] = m;
  }
  ap.count += (uint32_t)__popc(ib);
  const uint32_t ex = ev & ~ib;
  if (ex) ap.min_excl = umin64(ap.min_excl, g + (uint64_t)__builtin_ctz(ex));
  if (ev) ap.flags |= pk.miss;
  return ib;
}

// a read over the lag view (am_op_log.lag_ct / lag / key_lag): its key's lag bases
template <int DMAX>
struct LagRead {
  bool on;
  uint32_t lb[DMAX];
};
template <int DMAX>
__device__ __forceinline__ void lag_setup(const am_op_log &L, uint32_t nd, uint64_t key, bool on, LagRead<DMAX> &lr) {
  lr.on = on;
#pragma unroll
  for (int d = 0; d < DMAX; ++d) lr.lb[d] = on && d < (int)nd ? uniform_u32((uint32_t)L.key_lag[key * nd + d]) : 0u;
}

// pk_tile (am_wave.h) over the lag view: the OPL ops' commit entries c (AM_PK_ESC: escaped, or a
// lag beyond 16 bits) and their u16 lags lw (two per word), the entries X[d] - K = c - (lb[d] +
// lag) rebuilt where the compares and the max use them
template <int DMAX, int OPL, bool GENERAL>
__device__ __forceinline__ uint32_t pk_tile_lag(const ReadU<DMAX> &u, const PkRead<DMAX> &pk, const LagRead<DMAX> &lr,
                                                const uint32_t (&c)[OPL], const uint32_t (&lw)[DMAX][(OPL + 1) / 2],
                                                const uint64_t (&tx)[OPL], uint64_t g, uint64_t off0, uint64_t off1,
                                                AccP<DMAX> &ap, bool &esc) {
  auto xd = [&](int k, int d) -> uint32_t {
    const uint32_t w = lw[d][k / 2];
    return c[k] - (lr.lb[d] + ((k & 1) ? w >> 16 : w & 0xFFFFu));
  };
  uint32_t ib = 0, ev = 0;
#pragma unroll
  for (int k = 0; k < OPL; ++k) {
    const uint64_t p = g + k;
    const bool inr = p >= off0 && p < off1;
    const bool e = c[k] == AM_PK_ESC;
    esc |= inr && e;
    uint32_t over = 0;
#pragma unroll
    for (int d = 0; d < DMAX; ++d) over |= __builtin_elementwise_sub_sat(xd(k, d), pk.thr[d]);
    bool cand = inr && !e;
    if (GENERAL) {  // belongs_to_snapshot_op: not vectorclock:le(X, base)
      uint32_t cov = 0;
#pragma unroll
      for (int d = 0; d < DMAX; ++d) cov |= __builtin_elementwise_sub_sat(xd(k, d), pk.cthr[d]);
      const bool le = !pk.cnever && cov == 0;
      cand = cand && (u.base_ignore || (u.has_txid && tx[k] == u.txid) || !le);
    }
    ib |= (uint32_t)(cand && !pk.never && over == 0) << k;
    ev |= (uint32_t)cand << k;
  }
#pragma unroll
  for (int d = 0; d < DMAX; ++d) {
    uint32_t m = ap.mx[d];
#pragma unroll
    for (int k = 0; k < OPL; ++k) m = max(m, ((ib >> k) & 1u) ? xd(k, d) : 0u);
    ap.mx[d] = m;
  }
  ap.count += (uint32_t)__popc(ib);
  const uint32_t ex = ev & ~ib;
  if (ex) ap.min_excl = umin64(ap.min_excl, g + (uint64_t)__builtin_ctz(ex));
  if (ev) ap.flags |= pk.miss;
  return ib;
}

// Inclusion of the 4 ops [g, g + 4) of one read inside [lo, hi) (is_op_in_snapshot/7 +
// belongs_to_snapshot_op/3, every clock general): bit k = op g + k included.  Packed view
// (PACKED): u32 entries through pk_tile, partials in ap, escaped ops from the full columns;
// full view: eval_op on the u64 columns, partials in a.  AM_META_BAD ops are included here
// (eval_op flags them); callers skip their effects.
template <int DMAX, bool PACKED>
__device__ __forceinline__ uint32_t incl4(const am_op_log &L, uint32_t nd, uint64_t stride, const ReadU<DMAX> &u,
                                          const PkRead<DMAX> &pk, uint64_t g, uint64_t lo, uint64_t hi, AccP<DMAX> &ap,
                                          Acc<DMAX> &a) {
  uint64_t tx[4] = {0, 0, 0, 0};
  if (u.has_txid) {
    const u64x2 t01 = *(const u64x2 *)(L.op_txid + g), t23 = *(const u64x2 *)(L.op_txid + g + 2);
    tx[0] = t01.x, tx[1] = t01.y, tx[2] = t23.x, tx[3] = t23.y;
  }
  uint32_t ib = 0;
  bool esc = false;
  if (PACKED) {
    uint32_t x[4][DMAX];
#pragma unroll
    for (int d = 0; d < DMAX; ++d) {
      u32x4 q = {0, 0, 0, 0};
      if (d < (int)nd) q = *(const u32x4 *)(L.pk_vc + (uint64_t)d * stride + g);
      x[0][d] = q.x, x[1][d] = q.y, x[2][d] = q.z, x[3][d] = q.w;
    }
    ib = pk_tile<DMAX, 4, true>(u, pk, x, tx, g, lo, hi, ap, esc);
    if (!esc) return ib;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint64_t p = g + k;
    if (p < lo || p >= hi) continue;
    if (PACKED && L.pk_vc[p] != AM_PK_ESC) continue;
    uint64_t sv[DMAX], ct;
    uint32_t meta;
    esc_load<DMAX>(L, nd, stride, p, sv, ct, meta);
    const uint32_t sp = L.snap_pres ? L.snap_pres[p] : u.allmask;
    if (eval_op<DMAX, true>(u, meta, ct, sv, sp, u.has_txid && tx[k] == u.txid, p, a)) ib |= 1u << k;
  }
  return ib;
}

// base bounded-counter slot i of read r (P slots i < np, then the nd D slots): row r of the
// [n][np] / [n][nd] arrays, or at base.bc_off[r] (snapshot-cache bases in the value pool)
// the base snapshot's bounded-counter entry at slot i (P {From,To} at From*nd+To, D Id at
// np+Id): its (slot, value) pairs sit in the base CSR sorted by slot -- binary search
__device__ __forceinline__ int64_t bc_base(const am_read_batch &B, uint64_t r, uint32_t np, uint32_t nd, uint32_t i,
                                           uint32_t &pres) {
  (void)np, (void)nd;
  pres = 0;
  if (!B.base.set_off || !B.base.set_len) return 0;
  const uint64_t o = B.base.set_off[r];
  uint32_t lo = 0, hi = B.base.set_len[r];
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (B.base.set_a[o + mid] < (uint64_t)i) lo = mid + 1;
    else hi = mid;
  }
  if (lo < B.base.set_len[r] && B.base.set_a[o + lo] == (uint64_t)i) {
    pres = 1;
    return (int64_t)B.base.set_b[o + lo];
  }
  return 0;
}

// A bounded-counter result: the read's present slots as (slot, value) pairs, slot order (the P
// orddict, then D, each in key order), into its CSR range of the result -- GL lanes of a wave
// (lane gl of the group, the group's lanes at wave bits [gbit, gbit + GL)), every lane of the
// group in the call.  get(k, v) -> slot k's presence and value.  Returns the number of present
// slots; more than the read's capacity: nothing past it is written (AM_ERR_CAPACITY).
template <int GL, class Get>
__device__ __forceinline__ uint32_t bc_emit(const am_read_result &R, uint64_t r, uint32_t ns, uint32_t gl,
                                            uint32_t gbit, Get get) {
  const uint64_t o = R.value.set_off[r], cap = R.value.set_off[r + 1] - o;
  const uint64_t gm = GL >= 64 ? ~0ull : ((1ull << GL) - 1ull), lt = (1ull << gl) - 1ull;
  uint32_t cnt = 0;
  for (uint32_t k0 = 0; k0 < ns; k0 += GL) {
    const uint32_t k = k0 + gl;
    int64_t v = 0;
    const bool p = k < ns && get(k, v);
    const uint64_t m = (__ballot(p) >> gbit) & gm;
    const uint64_t pos = cnt + (uint32_t)__popcll(m & lt);
    if (p && pos < cap) {
      R.value.set_a[o + pos] = k;
      R.value.set_b[o + pos] = (uint64_t)v;
    }
    cnt += (uint32_t)__popcll(m);
  }
  return cnt;
}

// ---- per-type value reductions (apply_operations folds of commutative updates) ----
struct PnVal {  // antidote_crdt_counter_pn: integer sum, exact in 128 bits
  int64_t hi;
  uint64_t lo;
  __device__ void reset() { hi = 0, lo = 0; }
  __device__ void add(uint64_t p0, uint64_t) {
    const int64_t v = (int64_t)p0;
    add128(hi, lo, v < 0 ? -1 : 0, (uint64_t)v);
  }
};
struct LwwVal {  // antidote_crdt_register_lww: erlang:max over {Ts, Value}
  uint64_t ts, val;
  uint32_t has;
  __device__ void reset() { ts = 0, val = 0, has = 0; }
  __device__ void add(uint64_t p0, uint64_t p1) {
    const bool gt = !has || p0 > ts || (p0 == ts && p1 > val);
    ts = gt ? p0 : ts;
    val = gt ? p1 : val;
    has = 1;
  }
};

template <int TYPE>
struct ValOf;
template <>
struct ValOf<AM_PN> {
  using T = PnVal;
  static constexpr bool NEED_P1 = false;
};
template <>
struct ValOf<AM_LWW> {
  using T = LwwVal;
  static constexpr bool NEED_P1 = true;
};

// wave-uniform LWW max: row butterflies on (has, ts, val), then the four rows
__device__ __forceinline__ void wave_max_lww(LwwVal &v) {
#define S_(C)                                                                            \
  {                                                                                      \
    const uint64_t wts = dpp64<C>(v.ts), wval = dpp64<C>(v.val);                         \
    const uint32_t whas = dpp32<C>(v.has);                                               \
    const bool gt = whas && (!v.has || wts > v.ts || (wts == v.ts && wval > v.val));     \
    v.ts = gt ? wts : v.ts;                                                              \
    v.val = gt ? wval : v.val;                                                           \
    v.has |= whas;                                                                       \
  }
  AMK_ROW_STEPS(S_)
#undef S_
  LwwVal r;
  r.ts = lane_u64(v.ts, 0), r.val = lane_u64(v.val, 0), r.has = lane_u32(v.has, 0);
#pragma unroll
  for (int l = 16; l < 64; l += 16) {
    const uint64_t wts = lane_u64(v.ts, l), wval = lane_u64(v.val, l);
    const uint32_t whas = lane_u32(v.has, l);
    const bool gt = whas && (!r.has || wts > r.ts || (wts == r.ts && wval > r.val));
    r.ts = gt ? wts : r.ts;
    r.val = gt ? wval : r.val;
    r.has |= whas;
  }
  v = r;
}

__device__ __forceinline__ void row_max_lww(LwwVal &v) {
#define S_(C)                                                                        \
  {                                                                                  \
    const uint64_t wts = dpp64<C>(v.ts), wval = dpp64<C>(v.val);                     \
    const uint32_t whas = dpp32<C>(v.has);                                           \
    const bool gt = whas && (!v.has || wts > v.ts || (wts == v.ts && wval > v.val)); \
    v.ts = gt ? wts : v.ts;                                                          \
    v.val = gt ? wval : v.val;                                                       \
    v.has |= whas;                                                                   \
  }
  AMK_ROW_STEPS(S_)
#undef S_
}

}  // namespace amk
