// am_group.h -- the token-group tier of the add-wins set and the MV register
// (antidote_crdt_set_aw / antidote_crdt_register_mv update/2, folded by
// clocksi_materializer:apply_operations/4, src/clocksi_materializer.erl:113-121), and the
// ingestion-side builder of the token-group view it reads (include/antidote_mat.h).
//
// Closed form.  Both types apply their effects sequentially, oldest -> newest, but the
// final state has a closed form.  Call every token an effect inserts a BIRTH at the op's
// position p (AW {Elem, [Token], _} -> (elem, token); MV {Value, Token, _} -> (value,
// token)) and every token it drops a KILL at p (AW remove tokens, MV overridden tokens).
// The AW update is ToAdd ++ (Current -- ToRemove) and the MV update drops the overridden
// tokens before insert_sorted, so a kill never hits a birth of its own op, and
//     a token survives  <=>  its newest included birth is at or after its newest included kill
// per kill key (AW (elem, token), MV token).  Tokens are unique() binaries in antidote_crdt,
// so a kill key has one birth; keys whose log breaks that (a token born twice, or under two
// MV values) are left ungrouped by the builder and go to the var_data tiers (am_sets.hip).
//
// Builder (k_grp_build, one workgroup per key, at store creation / update): the key's
// births and kills are sorted by kill key in LDS; every distinct kill key is a GROUP; the
// groups are numbered in the reference's output order -- AW: elem ascending, then newest
// birth first and, within one op, the effect's token order (ToAdd ++ Current); MV: (value,
// token) ascending (insert_sorted) -- and each birth/kill becomes one u32 record
// op | kill << 16 | group << 17.
//
// Read (k_grp_row: one 16-lane row per short read; k_grp_wave: one wave per read, up to
// 1024 groups; k_grp_wg: one 512-thread workgroup per read, up to 2048 groups):
//   1. the read's ops stream in 1024-op tiles (packed view, 16-byte loads): is_op_in_snapshot/7
//      per op (am_wave.h eval_op) -> an LDS inclusion bitmap + the scalar outputs;
//   2. the read's records (4 B each) stream in: an included birth sets its group's BORN bit,
//      an included kill its KILLED bit (LDS atomicOr; the builder keeps only EFFECTIVE kills,
//      those after the group's birth -- a kill in the birth's own op or earlier never
//      removes it: ToAdd ++ (Current -- ToRemove), MV drops before inserting);
//   3. the groups are scanned in order: survivors (born and not killed) are compacted by
//      wave ballots and their (a, b) pairs gathered into the output CSR -- already in the
//      reference's order, no sort.
// Reads with base-snapshot pairs, longer logs or ungrouped keys are handed to the next tier.
#pragma once
#include "am_block.h"

namespace amk_grp {
using namespace amk;

// phase timing of the wave kernel (experiments only, -DAMK_PHASE_PROF): per-wave cycles
// spent from one phase boundary to the next, summed into amk_phase_cycles
#ifdef AMK_PHASE_PROF
__device__ unsigned long long amk_phase_cycles[8];
#define PH_BEGIN() uint64_t ph_t = clock64()
#define PH(i)                                   \
  {                                             \
    const uint64_t ph_n = clock64();            \
    ph_acc[i] += ph_n - ph_t;                   \
    ph_t = ph_n;                                \
  }
#define PH_END()                                                               \
  if ((threadIdx.x & 63) == 0)                                                 \
    for (int q = 0; q < 6; ++q) atomicAdd(&amk_phase_cycles[q], (unsigned long long)ph_acc[q])
#define PH_DECL() uint64_t ph_acc[6] = {0, 0, 0, 0, 0, 0}
#else
#define PH_BEGIN()
#define PH(i)
#define PH_END()
#define PH_DECL()
#endif
constexpr int BLOCK = 256;
constexpr int NW = BLOCK / WAVE;
constexpr uint32_t RCAP = AM_GRP_MAX_REC;
constexpr uint32_t KILL31 = 0x80000000u;

// ================================================================ reads
// per-read metadata shared by both read kernels
struct GMeta {
  uint64_t r, key, off0, off1, rk0, rk1;
  uint32_t G;
  int32_t st;
};

__device__ __forceinline__ void read_meta(const am_op_log &L, const am_read_batch &B, uint64_t r, uint32_t type,
                                          GMeta &m) {
  m.r = r;
  m.key = B.key[r];
  m.st = AM_OK;
  m.off0 = m.off1 = m.rk0 = m.rk1 = 0;
  m.G = AM_NGRP_NONE;
  const uint32_t rtype = B.type[r];
  if (m.key >= L.n_keys) {
    m.st = AM_ERR_INVALID;
    return;
  }
  m.off0 = L.key_off[m.key];
  m.off1 = am_kend(L, m.key);
  const uint32_t ktype = L.key_type[m.key];
  const uint32_t kfl = L.key_flags ? (uint32_t)L.key_flags[m.key] : 0u;
  if (m.off1 > m.off0 && (ktype != rtype || (kfl & AM_KEY_MIXED_TYPES))) m.st = AM_ERR_CORRUPTED_OPS_CACHE;
  else if (rtype != type) m.st = AM_ERR_INVALID;
  if (m.st != AM_OK) return;
  m.rk0 = L.rec_key_off[m.key];
  m.rk1 = am_rkend(L, m.key);
  m.G = L.key_ngrp[m.key];
}

__device__ __forceinline__ bool has_base_pairs(const am_read_batch &B, uint64_t r) {
  return B.base.set_off && B.base.set_len && B.base.set_len[r] != 0;
}

// per-read inputs (clock, base clock, TxId) of read r; UNIF: the whole workgroup reads one
// read, so the values are made wave-uniform (scalar registers)
template <int DMAX, bool GENERAL, bool UNIF>
__device__ __forceinline__ void read_inputs(const am_op_log &L, uint32_t nd, const am_read_batch &B, uint64_t r,
                                            ReadU<DMAX> &u) {
  auto u32 = [](uint32_t x) { return UNIF ? uniform_u32(x) : x; };
  auto u64 = [](uint64_t x) { return UNIF ? uniform_u64(x) : x; };
  const uint64_t n = B.n_reads;
  u.allmask = nd >= 32 ? 0xFFFFFFFFu : ((1u << nd) - 1u);
  const uint64_t rstride = (GENERAL && B.per_read_clock) ? n : 1, ridx = (GENERAL && B.per_read_clock) ? r : 0;
  u.spres = u32(B.read_pres[ridx]) & u.allmask;
  u.base_ignore = !GENERAL || !B.base_ignore || B.base_ignore[r];
  u.cpres = u.base_ignore ? 0u : (u32(B.base_pres[r]) & u.allmask);
#pragma unroll
  for (int d = 0; d < DMAX; ++d) {
    u.S[d] = (d < (int)nd && ((u.spres >> d) & 1u)) ? u64(B.read_vc[(uint64_t)d * rstride + ridx]) : 0;
    u.C0[d] = (d < (int)nd && ((u.cpres >> d) & 1u)) ? u64(B.base_vc[(uint64_t)d * n + r]) : 0;
  }
  u.has_txid = GENERAL && B.txid && (!B.txid_valid || B.txid_valid[r]) && L.op_txid;
  u.txid = u.has_txid ? u64(B.txid[r]) : 0;
}

// read_inputs (GENERAL, uniform) in two halves, so that a wave's NEXT read's inputs are in
// flight while it reads this one: in_load issues every load of read r at once as vector loads
// (lane d < nd: DC d's clock and base clock entries; lanes 0-4 one scalar each) -- the chain
// read_pres -> clock, base_ignore -> base_pres -> base clock, txid_valid -> txid is not
// waited on link by link -- and in_take builds the ReadU from them.  A base column is read
// whenever the batch has one (its [n_dc][n_reads] extent), its entries used only as
// read_inputs uses them.
struct InPre {
  uint64_t s, c, x;  // lane d: S[d] / C0[d] candidates; lane 4: the TxId
  uint32_t w;        // lane 0 read_pres, 1 base_ignore, 2 base_pres, 3 txid_valid
};
// Marks registers as used here: the compiler waits for their loads at this point (where the
// wave waits for older loads anyway) instead of at their real use, which can sit behind this
// read's output stores -- a wave's loads and stores retire through one counter (vmcnt), and a
// wait placed at a loop head cannot count them, so it would wait for every store.
template <typename T>
__device__ __forceinline__ void hold(const T &v) {
  asm volatile("" ::"v"(v));
}
__device__ __forceinline__ void hold(const InPre &p) { hold(p.s), hold(p.c), hold(p.x), hold(p.w); }

__device__ __forceinline__ void in_load(const am_op_log &L, uint32_t nd, const am_read_batch &B, uint64_t r,
                                        uint32_t lane, InPre &p) {
  const uint64_t n = B.n_reads;
  const bool prc = B.per_read_clock;
  p.s = p.c = p.x = 0, p.w = 0;
  if (lane < nd) {
    p.s = B.read_vc[prc ? (uint64_t)lane * n + r : (uint64_t)lane];
    if (B.base_ignore && B.base_vc) p.c = B.base_vc[(uint64_t)lane * n + r];
  }
  if (lane == 0) p.w = (uint32_t)B.read_pres[prc ? r : 0];
  if (lane == 1) p.w = B.base_ignore ? (uint32_t)B.base_ignore[r] : 1u;
  if (lane == 2 && B.base_ignore && B.base_pres) p.w = (uint32_t)B.base_pres[r];
  if (lane == 3) p.w = B.txid_valid ? (uint32_t)B.txid_valid[r] : 1u;
  if (lane == 4 && B.txid && L.op_txid) p.x = B.txid[r];
}
template <int DMAX>
__device__ __forceinline__ void in_take(const am_op_log &L, uint32_t nd, const am_read_batch &B, const InPre &p,
                                        ReadU<DMAX> &u) {
  u.allmask = nd >= 32 ? 0xFFFFFFFFu : ((1u << nd) - 1u);
  u.spres = lane_u32(p.w, 0) & u.allmask;
  u.base_ignore = !B.base_ignore || lane_u32(p.w, 1) != 0;
  u.cpres = u.base_ignore ? 0u : (lane_u32(p.w, 2) & u.allmask);
#pragma unroll
  for (int d = 0; d < DMAX; ++d) {
    u.S[d] = (d < (int)nd && ((u.spres >> d) & 1u)) ? lane_u64(p.s, d) : 0;
    u.C0[d] = (d < (int)nd && ((u.cpres >> d) & 1u)) ? lane_u64(p.c, d) : 0;
  }
  u.has_txid = B.txid && lane_u32(p.w, 3) != 0 && L.op_txid;
  u.txid = u.has_txid ? lane_u64(p.x, 4) : 0;
}

// N consecutive elements per lane (N = 1, 2 or a multiple of 4 / 2; 16-byte loads)
template <int N>
__device__ __forceinline__ void ld_n64(const uint64_t *p, uint64_t *o) {
  if constexpr (N == 1) {
    o[0] = *p;
  } else {
#pragma unroll
    for (int i = 0; i < N; i += 2) {
      const u64x2 a = *(const u64x2 *)(p + i);
      o[i] = a.x, o[i + 1] = a.y;
    }
  }
}
template <int N>
__device__ __forceinline__ void ld_n32(const uint32_t *p, uint32_t *o) {
  if constexpr (N >= 4) {
#pragma unroll
    for (int i = 0; i < N; i += 4) {
      const u32x4 a = *(const u32x4 *)(p + i);
      o[i] = a.x, o[i + 1] = a.y, o[i + 2] = a.z, o[i + 3] = a.w;
    }
  } else if constexpr (N == 2) {
    typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
    const u32x2_t a = *(const u32x2_t *)p;
    o[0] = a.x, o[1] = a.y;
  } else {
    o[0] = *p;
  }
}

// the OPL ops [g, g + OPL) of a read's [off0, off1): inclusion bits (is_op_in_snapshot/7).
// Packed view: u32 entries relative to the key's time base (am_wave.h pk_eval), partials in
// ap; an escaped op (pk_vc[0] == AM_PK_ESC) is not evaluated here: esc is set and the
// caller's escape pass (esc_pass) evaluates it from the full columns, off the hot loop.  With
// the lag view (lr.on) the same from 4 + 2 D bytes per op (escapes: lag_ct == AM_PK_ESC).
// Full view: eval_op on the u64 columns, partials in a.
template <int DMAX, int OPL, bool GENERAL, bool PACKED>
__device__ __forceinline__ uint32_t eval_tile(const am_op_log &L, uint32_t nd, const ReadU<DMAX> &u,
                                              const PkRead<DMAX> &pk, const LagRead<DMAX> &lr, uint64_t g,
                                              uint64_t off0, uint64_t off1, uint64_t stride, AccP<DMAX> &ap,
                                              Acc<DMAX> &a, bool &esc) {
  uint32_t ib = 0;
  uint64_t tx[OPL] = {};
  if (GENERAL && u.has_txid) ld_n64<OPL>(L.op_txid + g, tx);
  if (PACKED && lr.on) {
    uint32_t c[OPL] = {}, lw[DMAX][(OPL + 1) / 2];
    ld_n32<OPL>(L.lag_ct + g, c);
#pragma unroll
    for (int d = 0; d < DMAX; ++d) {
      const uint16_t *lp = L.lag + (uint64_t)d * stride + g;
      if constexpr (OPL == 4) {
        const uint2 v = d < (int)nd ? *(const uint2 *)lp : uint2{0, 0};
        lw[d][0] = v.x, lw[d][1] = v.y;
      } else if constexpr (OPL == 2) {
        lw[d][0] = d < (int)nd ? *(const uint32_t *)lp : 0u;
      } else {
        lw[d][0] = d < (int)nd ? (uint32_t)*lp : 0u;
      }
    }
    ib = pk_tile_lag<DMAX, OPL, GENERAL>(u, pk, lr, c, lw, tx, g, off0, off1, ap, esc);
  } else if (PACKED) {
    uint32_t x[OPL][DMAX];
#pragma unroll
    for (int d = 0; d < DMAX; ++d) {
      uint32_t q[OPL] = {};
      if (d < (int)nd) ld_n32<OPL>(L.pk_vc + (uint64_t)d * stride + g, q);
#pragma unroll
      for (int k = 0; k < OPL; ++k) x[k][d] = q[k];
    }
    ib = pk_tile<DMAX, OPL, GENERAL>(u, pk, x, tx, g, off0, off1, ap, esc);
  } else {
    uint64_t ct[OPL], sv[OPL][DMAX];
    uint32_t sp[OPL];
#pragma unroll
    for (int k = 0; k < OPL; ++k) sp[k] = u.allmask;
    if (GENERAL && L.snap_pres) ld_n32<OPL>(L.snap_pres + g, sp);
    ld_n64<OPL>(L.commit_time + g, ct);
    const uint32_t m4 = OPL == 4 ? *(const uint32_t *)(L.op_meta + g)
                        : OPL == 2 ? (uint32_t)*(const uint16_t *)(L.op_meta + g) : (uint32_t)L.op_meta[g];
#pragma unroll
    for (int d = 0; d < DMAX; ++d) {
      uint64_t q[OPL] = {};
      if (d < (int)nd) ld_n64<OPL>(L.snap_vc + (uint64_t)d * stride + g, q);
#pragma unroll
      for (int k = 0; k < OPL; ++k) sv[k][d] = q[k];
    }
#pragma unroll
    for (int k = 0; k < OPL; ++k) {
      const uint64_t p = g + k;
      if (p < off0 || p >= off1) continue;
      const uint32_t meta = (m4 >> (8 * k)) & 0xFFu;
      const bool txm = GENERAL && u.has_txid && tx[k] == u.txid;
      if (eval_op<DMAX, GENERAL>(u, meta, ct[k], sv[k], sp[k], txm, p, a) && !(meta & AM_META_BAD)) ib |= 1u << k;
    }
  }
  return ib;
}

// the escaped ops of ops [off0, off1) handled by this lane (p = off0 + lane0, step nl), from
// the full columns; included ones are OR-ed into the LDS bitmap (bit = p - t0)
template <int DMAX, bool GENERAL>
__device__ __forceinline__ void esc_pass(const am_op_log &L, uint32_t nd, const ReadU<DMAX> &u, uint64_t off0,
                                      uint64_t off1, uint64_t t0, uint64_t stride, uint32_t lane0, uint32_t nl,
                                      uint32_t *incl, Acc<DMAX> &a, const uint32_t *escv) {
  for (uint64_t p = off0 + lane0; p < off1; p += nl) {
    if (escv[p] != AM_PK_ESC) continue;
    uint64_t sv[DMAX], ct;
    uint32_t meta;
    esc_load<DMAX>(L, nd, stride, p, sv, ct, meta);
    const uint32_t sp = (GENERAL && L.snap_pres) ? L.snap_pres[p] : u.allmask;
    const bool txm = GENERAL && u.has_txid && L.op_txid[p] == u.txid;
    if (eval_op<DMAX, GENERAL>(u, meta, ct, sv, sp, txm, p, a) && !(meta & AM_META_BAD))
      atomicOr(&incl[(uint32_t)((p - t0) >> 5)], 1u << ((p - t0) & 31));
  }
}

// the same for a fresh read whose bits live in the global bitmap gbm (bit = op slot); escv: the
// view the read streamed (pk_vc, or the lag view's lag_ct), whose AM_PK_ESC marks the escapes
template <int DMAX>
__device__ void esc_pass_g(const am_op_log &L, uint32_t nd, const ReadU<DMAX> &u, uint64_t off0, uint64_t off1,
                           uint64_t stride, uint32_t lane, uint32_t *gbm, Acc<DMAX> &a, const uint32_t *escv) {
  for (uint64_t p = off0 + lane; p < off1; p += WAVE) {
    if (escv[p] != AM_PK_ESC) continue;
    uint64_t sv[DMAX], ct;
    uint32_t meta;
    esc_load<DMAX>(L, nd, stride, p, sv, ct, meta);
    if (eval_op<DMAX, false>(u, meta, ct, sv, u.allmask, false, p, a) && !(meta & AM_META_BAD))
      atomicOr(&gbm[p >> 5], 1u << (p & 31));
  }
}

// a wave's scalar outputs (in every lane): packed partials (u32, relative to K) and, when
// `full` (wave-uniform: the full view, or escaped ops), full-width partials.  mxl: lane d's
// max X[d] over the included ops (0 when none)
template <int DMAX, bool PACKED>
__device__ __forceinline__ void wave_scalars(const AccP<DMAX> &ap, const Acc<DMAX> &a, bool full, uint64_t K,
                                             uint32_t allmask, uint32_t nd, uint32_t lane, uint32_t &count,
                                             uint32_t &flags, uint32_t &pres, uint64_t &min_excl, uint64_t &mxl) {
  count = 0, flags = 0, pres = 0, mxl = 0;
  min_excl = wave_min_u64_v(umin64(ap.min_excl, a.min_excl));
  if (PACKED) {
    const uint32_t cp = wave_sum_u32_v(ap.count);
    count = cp, flags = wave_or_u32_v(ap.flags), pres = cp ? allmask : 0u;
#pragma unroll
    for (int d = 0; d < DMAX; ++d) {
      if (d >= (int)nd) continue;
      const uint32_t m = wave_max_u32_v(ap.mx[d]);
      if ((uint32_t)d == lane) mxl = cp ? K + m : 0;
    }
  }
  if (full) {
    count += wave_sum_u32_v(a.count), flags |= wave_or_u32_v(a.flags), pres |= wave_or_u32_v(a.pres);
#pragma unroll
    for (int d = 0; d < DMAX; ++d) {
      if (d >= (int)nd) continue;
      const uint64_t m = wave_max_u64_v(a.mx[d]);
      if ((uint32_t)d == lane) mxl = umax64(mxl, m);
    }
  }
}

// NewLastOp: id of the oldest excluded candidate - 1, else get_first_id/1 (the newest op's id)
__device__ __forceinline__ int64_t new_last_op(const am_op_log &L, uint64_t key, uint64_t off0, uint64_t off1,
                                               uint64_t min_excl) {
  const uint64_t idb = L.key_id_base ? L.key_id_base[key] : 1;
  if (min_excl != NONE) return (L.op_id ? (int64_t)L.op_id[min_excl] : (int64_t)(idb + (min_excl - off0))) - 1;
  if (off1 == off0) return 0;
  return L.op_id ? (int64_t)L.op_id[off1 - 1] : (int64_t)(idb + (off1 - off0) - 1);
}

// the same from the key's op-id base (key_id_base[key], or 1)
__device__ __forceinline__ int64_t new_last_op_b(const am_op_log &L, uint64_t idb, uint64_t off0, uint64_t off1,
                                                 uint64_t min_excl) {
  if (min_excl != NONE) return (L.op_id ? (int64_t)L.op_id[min_excl] : (int64_t)(idb + (min_excl - off0))) - 1;
  if (off1 == off0) return 0;
  return L.op_id ? (int64_t)L.op_id[off1 - 1] : (int64_t)(idb + (off1 - off0) - 1);
}

template <int DMAX>
__device__ __forceinline__ void write_scalars(const am_op_log &L, uint32_t nd, const am_read_batch &B, am_read_result &R,
                                              const GMeta &m, const ReadU<DMAX> &u, int32_t status, uint32_t count,
                                              uint32_t flags, uint32_t pres, uint64_t min_excl, const uint64_t *mx,
                                              uint32_t setlen) {
  const uint64_t r = m.r, n = B.n_reads;
  R.status[r] = status;
  R.flags[r] = (uint8_t)(flags & 0xFFu);
  if (status != AM_OK) return;
  R.new_last_op[r] = new_last_op(L, m.key, m.off0, m.off1, min_excl);
  const bool ign = u.base_ignore && count == 0;
  const uint32_t opres = ign ? 0u : (pres | u.cpres);
  R.last_ct_ignore[r] = ign ? 1 : 0;
  R.last_ct_pres[r] = opres;
#pragma unroll
  for (int d = 0; d < DMAX; ++d) {
    if (d >= (int)nd) continue;
    const uint64_t v = mx[d] > u.C0[d] ? mx[d] : u.C0[d];
    R.last_ct[(uint64_t)d * n + r] = ((opres >> d) & 1u) ? v : 0;
  }
  R.is_new_ss[r] = count > 0;
  R.count[r] = count;
  R.value.set_len[r] = setlen;
}

// ---------------------------------------------------------------- workgroup per read
// 512 threads: one 1024-op tile (2 ops per thread at D >= 8, 2048 ops / 4 per thread below)
// and 2048 records are in flight per read, with no register double-buffering; several
// workgroups per CU overlap one read's LDS phases with another's loads.
constexpr int WBLOCK = 512;
constexpr int WNW = WBLOCK / WAVE;
constexpr uint32_t OPMAX = 8192;                  // longest log of the workgroup kernel
constexpr uint32_t IWORDS = OPMAX / 32 + 64;      // + tile alignment slack
constexpr int RPT = 4;                            // records per thread per pass
constexpr uint64_t RPASS = (uint64_t)WBLOCK * RPT;
template <int DMAX>
constexpr int wopl() { return DMAX >= 8 ? 2 : 4; }

template <int DMAX>
struct WgSmem {
  uint32_t born[RCAP / 32], killed[RCAP / 32];  // per group: birth included / an effective kill included
  uint32_t incl[IWORDS];        // included ops, bit = op - (off0 & ~(OPL-1))
  uint64_t red[WNW][4 + DMAX];  // per-wave partials: count, flags, pres, min_excl, mx[]
  uint32_t wsum[WNW];
};

template <int DMAX, int TYPE, bool GENERAL, bool PACKED, bool EXACT>
__global__ void __launch_bounds__(WBLOCK, 4) k_grp_wg(am_op_log L, am_read_batch B, am_read_result R, am_sel S,
                                                      am_retry next) {
  constexpr int OPL = wopl<DMAX>();
  constexpr uint64_t TILE = (uint64_t)WBLOCK * OPL;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  WgSmem<DMAX> &s = *reinterpret_cast<WgSmem<DMAX> *>(smem_raw);
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint64_t lt = (1ull << lane) - 1ull;
  const uint32_t nd = EXACT ? (uint32_t)DMAX : L.n_dc;  // EXACT: n_dc == DMAX, no per-DC guards
  const uint64_t stride = L.snap_stride ? L.snap_stride : L.n_ops;
  const uint32_t sel0 = S.idx ? uniform_u32(S.range[0]) : 0u;
  const uint64_t nsel = S.idx ? (uint64_t)(uniform_u32(S.range[1]) - sel0) : B.n_reads;

  for (uint64_t i = blockIdx.x; i < nsel; i += gridDim.x) {
    GMeta m;
    read_meta(L, B, S.idx ? (uint64_t)uniform_u32(S.idx[sel0 + i]) : i, TYPE, m);
    m.st = (int32_t)uniform_u32((uint32_t)m.st);
    m.off0 = uniform_u64(m.off0), m.off1 = uniform_u64(m.off1);
    m.rk0 = uniform_u64(m.rk0), m.rk1 = uniform_u64(m.rk1), m.G = uniform_u32(m.G);
    const uint64_t r = m.r;
    if (m.st != AM_OK) {
      if (tid == 0) R.status[r] = m.st, R.flags[r] = 0;
      continue;
    }
    const uint32_t G = m.G;
    if (G == AM_NGRP_NONE || G > RCAP || m.off1 - m.off0 > OPMAX || has_base_pairs(B, r)) {
      if (tid == 0) next.list[atomicAdd(next.count, 1u)] = (uint32_t)r;
      continue;
    }
    ReadU<DMAX> u;
    read_inputs<DMAX, GENERAL, true>(L, nd, B, r, u);
    const uint64_t t0 = m.off0 & ~(uint64_t)(OPL - 1);
    const uint32_t sh = (uint32_t)(m.off0 & (OPL - 1));

    // the first record pass is in flight while the ops are evaluated
    uint32_t rec[RPT];
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
      const uint64_t q = m.rk0 + (uint64_t)j * WBLOCK + tid;
      rec[j] = q < m.rk1 ? L.rec_g[q] : 0xFFFFFFFFu;
    }
    for (uint32_t g = tid; g < (G + 31) / 32; g += WBLOCK) s.born[g] = 0, s.killed[g] = 0;

    // ---- 1. inclusion per op -> bitmap + scalar partials ----
    PkRead<DMAX> pk;
    if (PACKED) pk_setup(u, nd, uniform_u64(L.key_tbase[m.key]), pk);
    LagRead<DMAX> lr;
    lag_setup(L, nd, m.key, PACKED && L.lag_ct != nullptr, lr);
    AccP<DMAX> ap;
    Acc<DMAX> a;
    ap.reset();
    a.reset();
    bool esc = false;  // some op of this lane did not fit the packed view
    for (uint64_t t = t0; t < m.off1; t += TILE) {
      const uint64_t g = t + (uint64_t)tid * OPL;
      const uint32_t ib =
          g < m.off1 ? eval_tile<DMAX, OPL, GENERAL, PACKED>(L, nd, u, pk, lr, g, m.off0, m.off1, stride, ap, a, esc)
                     : 0u;
      // 32 / OPL lanes -> one bitmap word
      constexpr uint32_t LPW = 32 / OPL;
      uint32_t word = ib << (OPL * (lane % LPW));
#pragma unroll
      for (uint32_t x = 1; x < LPW; x <<= 1) word |= (uint32_t)__shfl_xor((int)word, (int)x);
      if (lane % LPW == 0) s.incl[(uint32_t)((t - t0) / 32) + tid / LPW] = word;
    }
    const bool full = !PACKED || __syncthreads_or(esc);
    if (PACKED && full)  // rare: ops outside the packed view, from the full columns
      esc_pass<DMAX, GENERAL>(L, nd, u, m.off0, m.off1, t0, stride, tid, WBLOCK, s.incl, a,
                              lr.on ? L.lag_ct : L.pk_vc);
    {  // wave partials of the scalar outputs (VGPR reductions: the scalar file is full)
      uint32_t cnt, fl, pr;
      uint64_t mn, mxl;
      wave_scalars<DMAX, PACKED>(ap, a, full, PACKED ? pk.K : 0, u.allmask, nd, lane, cnt, fl, pr, mn, mxl);
      if (lane == 0) s.red[w][0] = cnt, s.red[w][1] = fl, s.red[w][2] = pr, s.red[w][3] = mn;
      if (lane < nd) s.red[w][4 + lane] = mxl;
    }
    __syncthreads();

    // ---- 2. records of included ops -> newest birth / kill per group ----
    for (uint64_t q0 = m.rk0;;) {
#pragma unroll
      for (int j = 0; j < RPT; ++j) {
        const uint32_t x = rec[j];
        if (x == 0xFFFFFFFFu) continue;
        const uint32_t op = AM_REC_OP(x), bit = op + sh;
        if (!((s.incl[bit >> 5] >> (bit & 31)) & 1u)) continue;
        atomicOr(((x & AM_REC_KILL) ? s.killed : s.born) + (AM_REC_GRP(x) >> 5), 1u << (AM_REC_GRP(x) & 31));
      }
      q0 += RPASS;
      if (q0 >= m.rk1) break;
#pragma unroll
      for (int j = 0; j < RPT; ++j) {
        const uint64_t q = q0 + (uint64_t)j * WBLOCK + tid;
        rec[j] = q < m.rk1 ? L.rec_g[q] : 0xFFFFFFFFu;
      }
    }
    // the block's scalar outputs (partials were published before the barrier above)
    uint32_t count = 0, flags = 0, pres = 0;
    uint64_t min_excl = NONE;
#pragma unroll
    for (int v = 0; v < WNW; ++v) {
      count += (uint32_t)s.red[v][0];
      flags |= (uint32_t)s.red[v][1];
      pres |= (uint32_t)s.red[v][2];
      min_excl = s.red[v][3] < min_excl ? s.red[v][3] : min_excl;
    }
    const int32_t st0 = (flags & FLAG_BAD) ? AM_ERR_UNEXPECTED_OPERATION : AM_OK;
    __syncthreads();

    // ---- 3. survivors in group order -> the output CSR ----
    uint32_t ns = 0;
    if (st0 == AM_OK) {
      const uint64_t ooff = R.value.set_off[r], ocap = R.value.set_off[r + 1] - ooff;
      for (uint32_t g0 = 0; g0 < G; g0 += WBLOCK) {
        const uint32_t g = g0 + tid;
        bool alive = false;
        if (g < G) alive = ((s.born[g >> 5] & ~s.killed[g >> 5]) >> (g & 31)) & 1u;
        const uint64_t bm = __ballot(alive);
        if (lane == 0) s.wsum[w] = (uint32_t)__popcll(bm);
        __syncthreads();
        uint32_t woff = 0, total = 0;
#pragma unroll
        for (int v = 0; v < WNW; ++v) {
          if (v < (int)w) woff += s.wsum[v];
          total += s.wsum[v];
        }
        if (alive) {
          const uint64_t o = ns + woff + (uint32_t)__popcll(bm & lt);
          if (o < ocap) {
            const u64x2 ab = *(const u64x2 *)(L.grp + 2 * (m.rk0 + g));
            R.value.set_a[ooff + o] = ab.x;
            R.value.set_b[ooff + o] = ab.y;
          }
        }
        ns += total;
        __syncthreads();
      }
    }
    if (tid < 64) {  // wave 0: lane d owns LastOpCt entry d, lane 0 the rest
      const uint64_t ocap = R.value.set_off[r + 1] - R.value.set_off[r];
      const int32_t status = (st0 == AM_OK && ns > ocap) ? AM_ERR_CAPACITY : st0;
      const bool ign = u.base_ignore && count == 0;
      const uint32_t opres = ign ? 0u : (pres | u.cpres);
      if (status == AM_OK && lane < nd) {
        uint64_t mx = 0, c0 = 0;
#pragma unroll
        for (int v = 0; v < WNW; ++v) mx = s.red[v][4 + lane] > mx ? s.red[v][4 + lane] : mx;
#pragma unroll
        for (int d = 0; d < DMAX; ++d)
          if ((uint32_t)d == lane) c0 = u.C0[d];
        R.last_ct[(uint64_t)lane * B.n_reads + r] = ((opres >> lane) & 1u) ? (mx > c0 ? mx : c0) : 0;
      }
      if (lane == 0) {
        R.status[r] = status;
        R.flags[r] = (uint8_t)(flags & 0xFFu);
        if (status == AM_OK) {
          R.new_last_op[r] = new_last_op(L, m.key, m.off0, m.off1, min_excl);
          R.last_ct_ignore[r] = ign ? 1 : 0;
          R.last_ct_pres[r] = opres;
          R.is_new_ss[r] = count > 0;
          R.count[r] = count;
          R.value.set_len[r] = ns;
        }
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- wave per read
// The C3-class read (hundreds to thousands of ops, up to VG groups): each wave of a
// 256-thread workgroup runs its own reads with no workgroup barrier -- LDS is carved per
// wave (group slots + inclusion bitmap) -- so a CU keeps ~16 reads in flight and one read's
// dependent steps (metadata -> ops + records -> survivors' pairs) hide behind the others.
constexpr uint32_t VG = AM_GRP_MAX_REC;    // groups of a wave-kernel read
constexpr uint32_t VOPS = 8192;            // ops of a wave-kernel read
constexpr uint32_t VWORDS = VOPS / 32 + 16;
constexpr int VRPT = 8;                    // records per lane per chunk (512 per wave)
// per-read metadata of a wave's batch of WB reads, loaded lane-parallel into LDS, so a read
// starts with no dependent global load (key -> key_off / records / time base / output range)
constexpr uint32_t WB = 32;
struct WSlot {
  uint64_t off0, rk0, ooff, K, idb, boff, key;
  uint32_t r, nops, nrec, G, ocap, nb;
};
// base-snapshot reads (cached AW / MV bases): at most KB base pairs and KB new survivors,
// merged in LDS (the survivor list area; see k_grp_wave step 4b)
constexpr uint32_t KB = 120;
constexpr uint32_t VGB = VG / 2;  // groups of a read whose survivors come through their births
struct WaveSmem {
  uint32_t born[VG / 32], killed[VG / 32];
  uint32_t incl[VWORDS];
  uint16_t list[VG];  // surviving groups in order
  uint16_t bri[VGB];  // per group (G <= VGB, every record streamed): its birth record from rk0
  WSlot slot[WB];
};
// ops per lane of a wave-kernel tile: the packed view's u32 entries fill 32-64 VGPRs; the
// full view's u64 columns 2 ops at D >= 8
template <int DMAX, bool PACKED>
constexpr int vopl() {
  return PACKED ? (DMAX <= 8 ? 4 : DMAX <= 16 ? 2 : 1) : (DMAX < 8 ? 4 : DMAX <= 16 ? 2 : 1);
}

// A read the wave kernel can take with its base snapshot: no base pairs, or at most KB of
// them and TxId ignore (an op of the reading transaction is a candidate even when the base
// holds it, and re-applying it duplicates tokens outside the closed form)
__device__ __forceinline__ bool base_ok(const am_op_log &L, const am_read_batch &B, uint64_t r) {
  if (!has_base_pairs(B, r)) return true;
  const bool txid = B.txid && (!B.txid_valid || B.txid_valid[r]) && L.op_txid;
  return !txid && B.base.set_len[r] <= KB;
}

// The wave tier takes a read (metadata mm, status ok): grouped within the LDS limits, its base
// acceptable, and not a short read the lane tier takes next (short_opl != 0).  The inclusion
// pass and the record pass of the split read (k_grp_incl, k_grp_wave<BM>) use the same test.
__device__ __forceinline__ bool wave_takes(const am_op_log &L, const am_read_batch &B, const GMeta &mm,
                                           uint32_t short_opl) {
  return !(mm.G == AM_NGRP_NONE || mm.G > VG || mm.off1 - mm.off0 > VOPS || !base_ok(L, B, mm.r) ||
           (short_opl && mm.G <= 64 && mm.off1 - (mm.off0 & ~(uint64_t)(short_opl - 1)) <= 64 &&
            !has_base_pairs(B, mm.r)));
}

// key order of the merge: AW elem (a); MV (value, token) (a, b)
template <int TYPE>
__device__ __forceinline__ bool key_lt(uint64_t a0, uint64_t b0, uint64_t a1, uint64_t b1) {
  return TYPE == AM_AWSET ? a0 < a1 : (a0 < a1 || (a0 == a1 && b0 < b1));
}

// The group of a base pair (AW (elem, token); MV token, under its value or ~0 when the log
// holds no birth of it), or ~0u.  Groups are ordered AW: elem, then newest birth first, unborn
// last; MV: (value | ~0, token).
template <int TYPE>
__device__ __forceinline__ uint32_t base_group(const am_op_log &L, uint64_t rk0, uint32_t G, uint64_t a, uint64_t b) {
  auto ga = [&](uint32_t g) { return L.grp[2 * (rk0 + g)]; };
  auto gb = [&](uint32_t g) { return L.grp[2 * (rk0 + g) + 1]; };
  if (TYPE == AM_AWSET) {
    uint32_t lo = 0, hi = G;  // first group with elem >= a
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (ga(mid) < a) lo = mid + 1;
      else hi = mid;
    }
    for (uint32_t g = lo; g < G; g += 4) {  // the elem's groups, four loads in flight
      u64x2 q[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) q[k] = g + k < G ? *(const u64x2 *)(L.grp + 2 * (rk0 + g + k)) : u64x2{~0ull, 0};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (q[k].x != a) return ~0u;
        if (q[k].y == b) return g + k;
      }
    }
    return ~0u;
  }
  for (int pass = 0; pass < 2; ++pass) {  // (value, token), then (~0, token)
    const uint64_t ka = pass ? ~0ull : a;
    uint32_t lo = 0, hi = G;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      const uint64_t x = ga(mid), y = gb(mid);
      if (x < ka || (x == ka && y < b)) lo = mid + 1;
      else hi = mid;
    }
    if (lo < G && ga(lo) == ka && gb(lo) == b) return lo;
  }
  return ~0u;
}

// a snapshot-cache read's group hints and pool tee (am_ctx::grp_hint_in, tee_*)
struct GrpHint {
  const uint32_t *in;  // [base word] the pair's group when it was cached, or null
  uint64_t *pa, *pb;   // the pool's words (null: no tee)
  uint32_t *pg;
  int64_t shift;       // pool word of result word o
  uint8_t *done;       // [read] its words are in the pool
  unsigned long long *skipped;  // the context's counters from AM_STAT_OPS_SKIPPED (am_ctx_stat)
  __device__ __forceinline__ void put(uint64_t o, uint64_t a, uint64_t b, uint32_t g) const {
    if (pa) {
      const uint64_t q = (uint64_t)((int64_t)o + shift);
      pa[q] = a, pb[q] = b, pg[q] = g;
    }
  }
};

// base pair (a, b)'s group through its hint: one load of the hinted group's pair; a hint
// whose pair does not match (the log changed since the snapshot was cached, or a tier that
// writes no hints produced the snapshot) falls back to the search.  Groups have distinct kill
// keys (AW (elem, token), MV token), so a matching pair is the group base_group finds.
template <int TYPE>
__device__ __forceinline__ uint32_t hinted_group(const am_op_log &L, uint64_t rk0, uint32_t G, uint64_t a, uint64_t b,
                                                 uint32_t hint) {
  if (hint < G) {
    const u64x2 q = *(const u64x2 *)(L.grp + 2 * (rk0 + hint));
    if (q.y == b && (q.x == a || (TYPE == AM_MVREG && q.x == ~0ull))) return hint;
  }
  return base_group<TYPE>(L, rk0, G, a, b);
}

// Step 4b of k_grp_wave: the read's value from a cached base.  materialize/4 folds the
// included candidates (ops not in the base, src/clocksi_materializer.erl:216-268) over the
// base state in log order; in closed form (causal logs: a remove follows the add it observed)
//   AW  per elem: [new tokens alive, newest first] ++ [base tokens not killed]   (ToAdd ++ (Current -- ToRemove))
//   MV  sorted union of the new pairs alive and the base pairs not overridden   (insert_sorted)
// where a base token is killed by an included candidate kill of its group (the builder keeps
// the kills of groups with no birth in the log: tokens a base holds from pruned ops).  The
// new survivors (<= KB) and the base pairs (<= KB) are listed in LDS (keys only) and each
// output position is its rank in its own list plus a binary-search count in the other.
// Returns false (nothing written) when the new survivors exceed KB.
template <int TYPE>
__device__ bool base_merge(const am_op_log &L, const am_read_batch &B, am_read_result &R, GrpHint H, WaveSmem &s,
                           uint64_t rk0, uint32_t G, uint32_t nb, uint64_t boff, uint64_t ooff, uint32_t ocap,
                           uint32_t lane, uint32_t &nout, int32_t &status, bool by_birth) {
  const uint32_t nwd = (G + 31) / 32;
  const uint32_t aw = lane < nwd ? (s.born[lane] & ~s.killed[lane]) : 0u;
  const uint32_t c = (uint32_t)__popc(aw);
  const uint32_t inc = wave_incl_scan_u32(c, lane);
  const uint32_t ns = (uint32_t)__shfl((int)inc, 63, WAVE);
  if (ns > KB) return false;
  // LDS: the survivor list area holds list[KB] u16 | nka[KB] nkb[KB] bka[KB] bkb[KB] u64
  uint16_t *list = s.list;
  uint64_t *nka = reinterpret_cast<uint64_t *>(s.list + KB), *nkb = nka + KB, *bka = nkb + KB, *bkb = bka + KB;
  static_assert(KB * 2 + 4 * KB * 8 <= VG * 2 && (KB * 2) % 8 == 0, "base-merge lists fit the survivor list area");
  uint64_t *balive = reinterpret_cast<uint64_t *>(s.incl);  // 2 words: base pairs alive
  {
    uint32_t o = inc - c;
    for (uint32_t bits = aw; bits; bits &= bits - 1) list[o++] = (uint16_t)(lane * 32 + __builtin_ctz(bits));
  }
  wave_sync();
  // new survivors' pairs (lanes i, i + 64) and keys
  u64x2 np[2] = {{0, 0}, {0, 0}};
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t i = lane + 64u * h;
    if (i < ns) {
      np[h] = by_birth ? *(const u64x2 *)(L.prec + 2 * (rk0 + s.bri[list[i]]))  // through its birth record
                 : *(const u64x2 *)(L.grp + 2 * (rk0 + list[i]));
      nka[i] = np[h].x, nkb[i] = np[h].y;
    }
  }
  // base pairs (lanes j, j + 64): alive unless an included candidate killed their group
  u64x2 bp[2] = {{0, 0}, {0, 0}};
  uint32_t bg[2] = {~0u, ~0u};
  uint64_t am[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t jb = lane + 64u * h;
    bool alive = false;
    if (jb < nb) {
      bp[h].x = B.base.set_a[boff + jb], bp[h].y = B.base.set_b[boff + jb];
      bka[jb] = bp[h].x, bkb[jb] = bp[h].y;
      const uint32_t g = H.in ? hinted_group<TYPE>(L, rk0, G, bp[h].x, bp[h].y, H.in[boff + jb])
                              : base_group<TYPE>(L, rk0, G, bp[h].x, bp[h].y);
      alive = g == ~0u || !((s.killed[g >> 5] >> (g & 31)) & 1u);
      bg[h] = g;
    }
    am[h] = __ballot(alive);
  }
  if (lane == 0) balive[0] = am[0], balive[1] = am[1];
  const uint32_t nbs = (uint32_t)(__popcll(am[0]) + __popcll(am[1]));
  wave_sync();
  nout = ns + nbs;
  if (nout > ocap) {
    status = AM_ERR_CAPACITY;
    return true;
  }
  // alive base pairs among the first x
  auto alive_below = [&](uint32_t x) -> uint32_t {
    const uint64_t a0 = balive[0], a1 = balive[1];
    if (x <= 64) return (uint32_t)__popcll(x == 64 ? a0 : (a0 & ((1ull << x) - 1ull)));
    return (uint32_t)__popcll(a0) + (uint32_t)__popcll(x - 64 == 64 ? a1 : (a1 & ((1ull << (x - 64)) - 1ull)));
  };
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t i = lane + 64u * h;
    if (i < ns) {  // + alive base pairs with a smaller key (AW ties: the new tokens first)
      uint32_t lo = 0, hi = nb;
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (key_lt<TYPE>(bka[mid], bkb[mid], np[h].x, np[h].y)) lo = mid + 1;
        else hi = mid;
      }
      const uint64_t o = ooff + i + alive_below(lo);
      R.value.set_a[o] = np[h].x, R.value.set_b[o] = np[h].y;
      H.put(o, np[h].x, np[h].y, list[i]);
    }
    const uint32_t jb = lane + 64u * h;
    if (jb < nb && ((am[h] >> lane) & 1ull)) {  // + new survivors with a key not above it
      uint32_t lo = 0, hi = ns;
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (!key_lt<TYPE>(bp[h].x, bp[h].y, nka[mid], nkb[mid])) lo = mid + 1;
        else hi = mid;
      }
      const uint64_t o = ooff + alive_below(jb) + lo;
      R.value.set_a[o] = bp[h].x, R.value.set_b[o] = bp[h].y;
      H.put(o, bp[h].x, bp[h].y, bg[h]);
    }
  }
  wave_sync();
  return true;
}

// BM (the split fresh read, after k_grp_incl): the inclusion bits come from the global bitmap
// ibm (bit p = op slot p) and the scalar outputs are already written; this pass streams the
// records and gathers the survivors only.
#ifndef AM_WAVE_FRESH_LAG
#define AM_WAVE_FRESH_LAG 0
#endif
#ifndef AM_WAVE_ZONE_LAG
#define AM_WAVE_ZONE_LAG 0
#endif
#ifndef AM_WAVE_WAVES
#define AM_WAVE_WAVES 4  // waves per SIMD the wave tier is compiled for
#endif
template <int DMAX, int TYPE, bool GENERAL, bool PACKED, bool EXACT, bool BM = false>
__global__ void __launch_bounds__(BLOCK, AM_WAVE_WAVES) k_grp_wave(am_op_log L, am_read_batch B, am_read_result R,
                                                                  am_sel S, am_retry next, uint32_t short_opl,
                                                                  GrpHint H, const uint32_t *ibm = nullptr) {
  constexpr int OPL = vopl<DMAX, PACKED>();
  constexpr uint64_t TILE = (uint64_t)WAVE * OPL;
  constexpr uint32_t LPW = 32 / OPL;  // lanes per bitmap word
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  WaveSmem &s = reinterpret_cast<WaveSmem *>(smem_raw)[threadIdx.x >> 6];
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  const uint64_t lt = (1ull << lane) - 1ull;
  const uint32_t nd = EXACT ? (uint32_t)DMAX : L.n_dc;
  const uint64_t stride = L.snap_stride ? L.snap_stride : L.n_ops;
  const uint32_t sel0 = S.idx ? uniform_u32(S.range[0]) : 0u;
  const uint64_t nsel = S.idx ? (uint64_t)(uniform_u32(S.range[1]) - sel0) : B.n_reads;
  const uint64_t W = (uint64_t)gridDim.x * NW;
  const uint64_t gw = (uint64_t)blockIdx.x * NW + uniform_u32(threadIdx.x >> 6);
  ReadU<DMAX> u;
  if (!GENERAL) read_inputs<DMAX, false, true>(L, nd, B, 0, u);  // one clock, no bases / TxIds
  uint64_t n_skipped = 0;  // ops of zones inside a base snapshot (uniform)
  uint64_t n_rskip = 0, n_gsw = 0;  // records not streamed, summary words read (uniform)
  PH_DECL();
  PH_BEGIN();

  for (uint64_t b0 = gw * WB; b0 < nsel; b0 += (uint64_t)WB * W) {
    // ---- lane j < WB: read b0 + j -> slot j (errors and hand-offs leave here).  A wave takes
    //      consecutive reads: its single-lane output stores fill whole lines of the columns ----
    const uint64_t ii = b0 + lane;
    bool elig = false, hand = false;
    uint64_t rr = 0;
    if (lane < WB && ii < nsel) {
      GMeta mm;
      read_meta(L, B, S.idx ? (uint64_t)S.idx[sel0 + ii] : ii, TYPE, mm);
      rr = mm.r;
      if (mm.st != AM_OK) {
        if (!BM) R.status[mm.r] = mm.st, R.flags[mm.r] = 0;
      } else if (!wave_takes(L, B, mm, short_opl)) {
        hand = !BM;  // (short_opl: a short read the lane tier takes next; BM: handed on by k_grp_incl)
      } else if (BM && R.status[mm.r] != AM_OK) {
        // the inclusion pass ended the read (an invalid effect included)
      } else {
        elig = true;
        WSlot &w = s.slot[lane];
        const uint64_t o0 = R.value.set_off[mm.r], o1 = R.value.set_off[mm.r + 1];
        w.off0 = mm.off0, w.rk0 = mm.rk0, w.ooff = o0;
        w.K = PACKED ? L.key_tbase[mm.key] : 0;
        w.key = mm.key;
        w.idb = L.key_id_base ? L.key_id_base[mm.key] : 1;
        w.r = (uint32_t)mm.r, w.nops = (uint32_t)(mm.off1 - mm.off0), w.nrec = (uint32_t)(mm.rk1 - mm.rk0);
        w.G = mm.G, w.ocap = o1 - o0 < 0xFFFFFFFFull ? (uint32_t)(o1 - o0) : 0xFFFFFFFFu;
        const bool hb = has_base_pairs(B, mm.r);
        w.nb = hb ? B.base.set_len[mm.r] : 0u;
        w.boff = hb ? B.base.set_off[mm.r] : 0;
      }
    }
    const uint64_t hm = __ballot(hand);
    if (hm) {
      uint32_t base = 0;
      if (lane == 0) base = atomicAdd(next.count, (uint32_t)__popcll(hm));
      base = uniform_u32(base);
      if (hand) next.list[base + (uint32_t)__popcll(hm & lt)] = (uint32_t)rr;
    }
    wave_sync();
    InPre ip{};  // GENERAL: the next read's inputs, in flight
    uint64_t em0 = __ballot(elig);
    if (GENERAL && em0) in_load(L, nd, B, uniform_u32(s.slot[__builtin_ctzll(em0)].r), lane, ip), hold(ip);

    for (uint64_t em = em0; em; em &= em - 1) {
      const uint32_t j = (uint32_t)__builtin_ctzll(em);
      const uint64_t off0 = uniform_u64(s.slot[j].off0), rk0 = uniform_u64(s.slot[j].rk0);
      const uint64_t off1 = off0 + uniform_u32(s.slot[j].nops), rk1 = rk0 + uniform_u32(s.slot[j].nrec);
      const uint64_t r = uniform_u32(s.slot[j].r);
      const uint32_t G = uniform_u32(s.slot[j].G);
      if (GENERAL) {
        in_take<DMAX>(L, nd, B, ip, u);
        const uint64_t rest = em & (em - 1);
        if (rest) in_load(L, nd, B, uniform_u32(s.slot[__builtin_ctzll(rest)].r), lane, ip);
      }
      // fresh reads over an exact-zone index stream tiles aligned to the zone blocks (a tile that
      // is one exact block is taken whole); the first tile masks the slots before off0
      const bool zal = !BM && !GENERAL && PACKED && TILE == AM_ZONE_OPS && L.zone_vc && off1 - off0 >= AM_ZONE_OPS;
      const uint64_t t0 = off0 & ~(uint64_t)((BM ? 32 : zal ? AM_ZONE_OPS : OPL) - 1);
      const uint32_t sh = (uint32_t)(off0 - t0);

      // the first record chunk is in flight while the ops are evaluated (loaded after the zone
      // test below).  A chunk is 512 records from the 16-byte-aligned qa: lane l holds records
      // qa + 4 l + 256 j + {0..3} (two 16-byte loads; records outside [rk0, rk1) are masked when
      // applied, and records re-applied are idempotent ORs)
      uint64_t qa = rk0 & ~3ull;
      // records [qs, qe) are not streamed: their blocks' group summaries stood in for them (fresh),
      // or their blocks are inside the base snapshot (cached: no included op)
      uint64_t qs = ~0ull, qe = 0;
      u32x4 rec[VRPT / 4];
      for (uint32_t g = lane; g < (G + 31) / 32; g += WAVE) s.born[g] = 0, s.killed[g] = 0;

      PH(0);
      // ---- 1. inclusion per op -> the wave's bitmap + per-lane scalar partials ----
      PkRead<DMAX> pk;
      if (PACKED) pk_setup(u, nd, uniform_u64(s.slot[j].K), pk);
      // the lag view (4 + 2 D bytes per op instead of 4 D): the cached (GENERAL) reads of a store
      // without a zone index.  Not the fresh variant (128 VGPRs: its lag branch spilled 39, the
      // indexed fresh C3 read 4.3 -> 6.4 ms) nor zone-indexed reads (their exact zones skip most
      // commit vectors; the per-read lag bases are one more dependent load round)
      LagRead<DMAX> lr;
      lag_setup(L, nd, uniform_u64(s.slot[j].key),
                PACKED && (GENERAL || AM_WAVE_FRESH_LAG) && L.lag_ct != nullptr && (AM_WAVE_ZONE_LAG || !L.zone_vc),
                lr);
      AccP<DMAX> ap;
      Acc<DMAX> a;
      ap.reset();
      a.reset();
      bool esc = false;  // some op of this lane did not fit the packed view
      // zone map: with a base snapshot (and no TxId), a tile whose zones are vectorclock:le the
      // base clock holds no candidate (belongs_to_snapshot_op/3) -- not streamed
      const bool zskip = !BM && GENERAL && L.zone_vc && !u.base_ignore && !u.has_txid;
      const uint64_t nz = (stride + AM_ZONE_OPS - 1) / AM_ZONE_OPS;
      // the read's zones in one round of loads: lane (d, z) tests zone z of DC d against the
      // base clock; a zone is inside the base when every DC's lane passes (reads spanning more
      // zones than a wave holds test per tile)
      uint64_t zin = 0;  // bit z - zb: zone z inside the base
      const uint64_t zb = t0 / AM_ZONE_OPS, nzr = (zskip && off1 > t0) ? (off1 - 1) / AM_ZONE_OPS - zb + 1 : 0;
      const bool zbatch = zskip && nzr * nd <= (uint64_t)WAVE;
      if (zbatch) {
        // rows nd .. nd + 3 in the same round when they fit: the first run of zones inside the
        // base that are exact zones of a grouped key (records begin / end) hold no included op,
        // so their records are not streamed either
        const bool rrows = L.zone_gsum && nzr * (nd + 4) <= (uint64_t)WAVE;
        const uint32_t dl = lane / (uint32_t)nzr, zl = lane % (uint32_t)nzr;
        bool ok = true;
        uint64_t zr = 0;
        if (dl < nd) {
          uint64_t c0 = 0;
#pragma unroll
          for (int d = 0; d < DMAX; ++d) c0 = (uint32_t)d == dl ? u.C0[d] : c0;
          ok = L.zone_vc[(uint64_t)dl * nz + zb + zl] <= c0;
        } else if (rrows && dl <= nd + 3) {
          zr = L.zone_vc[(uint64_t)dl * nz + zb + zl];
        }
        const uint64_t okm = __ballot(ok);
        zin = nzr >= 64 ? ~0ull : ((1ull << nzr) - 1ull);
        for (uint32_t d = 0; d < nd; ++d) zin &= okm >> (d * nzr);
        if (rrows) {
          const uint64_t em = __ballot(dl == nd && zr == 1) >> (nd * nzr);
          const uint64_t vm = __ballot(dl == nd + 1 && zr != ~0ull) >> ((nd + 1) * nzr);
          const uint64_t f = zin & em & vm;
          if (f) {
            const uint32_t za = (uint32_t)__builtin_ctzll(f);
            const uint32_t P = ~(f >> za) == 0 ? 64u - za : (uint32_t)__builtin_ctzll(~(f >> za));
            qs = shfl_u64(zr, (nd + 3) * (uint32_t)nzr + za);
            qe = shfl_u64(zr, (nd + 2) * (uint32_t)nzr + za + P - 1);
          }
        }
      }
      // fresh reads (the batch clock): an aligned tile that is one EXACT zone whose bound the
      // clock covers includes every op -- its bits, count and LastOpCt maxima come from the zone,
      // not from the ops' commit vectors.  One round of loads per read: lane (d, z) tests zone z's
      // bound of DC d (row nd: the exactness mark)
      uint64_t zfull = 0;  // bit z - t0 / AM_ZONE_OPS: tile z is such a zone
      uint64_t zval = 0;   // this lane's bound (row d < nd)
      uint32_t zrows = 0;
      if (zal && !pk.never && off1 >= t0 + AM_ZONE_OPS) {
        zrows = (uint32_t)((off1 - t0) / AM_ZONE_OPS);  // the read's whole tiles
        if (zrows * (nd + 1) <= WAVE) {
          // rows nd + 1 .. nd + 3 (group-summary offset, records end / begin) in the same round
          // when they fit
          const uint32_t rows = (L.zone_gsum && zrows * (nd + 4) <= WAVE) ? nd + 4 : nd + 1;
          const uint32_t dl = lane / zrows, zl = lane % zrows;
          bool ok = true;
          if (dl < rows) {
            zval = L.zone_vc[(uint64_t)dl * nz + t0 / AM_ZONE_OPS + zl];
            uint64_t s0 = 0;
#pragma unroll
            for (int d = 0; d < DMAX; ++d) s0 = (uint32_t)d == dl ? u.S[d] : s0;
            ok = dl > nd || (dl == nd ? zval == 1 : zval <= s0);
          }
          const uint64_t okm = __ballot(ok);
          zfull = zrows >= 64 ? ~0ull : ((1ull << zrows) - 1ull);
          for (uint32_t d = 0; d <= nd; ++d) zfull &= okm >> (d * zrows);
          // the first run of whole zones with group summaries: their born / killed words come
          // from the summaries and their records are not streamed
          const uint64_t hm = __ballot(dl == nd + 1 && zval != ~0ull) >> ((nd + 1) * zrows);
          const uint64_t f = rows > nd + 1 ? zfull & hm : 0ull;
          if (f) {
            const uint32_t za = (uint32_t)__builtin_ctzll(f);
            const uint32_t P = ~(f >> za) == 0 ? 64u - za : (uint32_t)__builtin_ctzll(~(f >> za));
            const uint32_t gw = (G + 31) / 32;
            uint32_t bw = 0, kw = 0;
            for (uint32_t z = za; z < za + P; ++z) {
              const uint64_t o = shfl_u64(zval, (nd + 1) * zrows + z);
              if (lane < gw) bw |= L.zone_gsum[o + lane], kw |= L.zone_gsum[o + gw + lane];
            }
            if (lane < gw) s.born[lane] = bw, s.killed[lane] = kw;
            qs = shfl_u64(zval, (nd + 3) * zrows + za);
            qe = shfl_u64(zval, (nd + 2) * zrows + za + P - 1);
            n_gsw += (uint64_t)P * 2 * gw;
          }
        } else {
          zrows = 0;
        }
      }
      // survivors' pairs through their birth records (prec, births in op order: the survivors'
      // lie close together) when every record is streamed and the groups fit bri
      const bool by_birth = L.prec != nullptr && G <= VGB && !(qe > qs);
      if (qe > qs) {  // records not streamed; a leading range moves the stream's start
        n_rskip += qe - qs;
        if (qs <= rk0) qa = qe & ~3ull, qs = ~0ull;
      }
#pragma unroll
      for (int jj = 0; jj < VRPT / 4; ++jj) {
        const uint64_t q = qa + (uint64_t)jj * 4 * WAVE + 4 * lane;
        rec[jj] = q < rk1 ? *(const u32x4 *)(L.rec_g + q) : u32x4{~0u, ~0u, ~0u, ~0u};
      }
      if (BM) {  // the inclusion pass's bits of [t0, off1), word-aligned
        const uint32_t nw = (uint32_t)((off1 - t0 + 31) / 32);
        for (uint32_t i = lane; i < nw; i += WAVE) s.incl[i] = ibm[(t0 >> 5) + i];
      }
      for (uint64_t t = t0; !BM && t < off1; t += TILE) {
        const uint64_t g = t + (uint64_t)lane * OPL;
        if (!GENERAL && zfull) {
          const uint32_t zi = (uint32_t)((t - t0) / AM_ZONE_OPS);
          if ((zfull >> zi) & 1ull) {  // every op of the tile included
            if (lane % LPW == 0) s.incl[(uint32_t)((t - t0) / 32) + lane / LPW] = 0xFFFFFFFFu;
            if (lane == 0) ap.count += AM_ZONE_OPS;
#pragma unroll
            for (int d = 0; d < DMAX; ++d)
              if (d < (int)nd) {
                const uint64_t zm = shfl_u64(zval, (uint32_t)d * zrows + zi);
                ap.mx[d] = max(ap.mx[d], (uint32_t)(zm - pk.K));
              }
            n_skipped += AM_ZONE_OPS;
            continue;
          }
        }
        if (zskip) {
          const uint64_t te = t + TILE < off1 ? t + TILE : off1;
          const uint64_t z0 = t / AM_ZONE_OPS, z1 = (te - 1) / AM_ZONE_OPS;
          bool in_base = true;
          if (zbatch) {
            for (uint64_t z = z0; z <= z1; ++z) in_base &= (zin >> (z - zb)) & 1ull;
          } else {
            for (uint64_t z = z0; z <= z1; ++z)
#pragma unroll
              for (int d = 0; d < DMAX; ++d)
                if (d < (int)nd) in_base &= L.zone_vc[(uint64_t)d * nz + z] <= u.C0[d];
          }
          if (in_base) {
            if (lane % LPW == 0) s.incl[(uint32_t)((t - t0) / 32) + lane / LPW] = 0u;
            n_skipped += te - (t > off0 ? t : off0);
            continue;
          }
        }
        const uint32_t ib =
            g < off1 ? eval_tile<DMAX, OPL, GENERAL, PACKED>(L, nd, u, pk, lr, g, off0, off1, stride, ap, a, esc) : 0u;
        uint32_t word = ib << (OPL * (lane % LPW));
#pragma unroll
        for (uint32_t x = 1; x < LPW; x <<= 1) word |= (uint32_t)__shfl_xor((int)word, (int)x);
        if (lane % LPW == 0) s.incl[(uint32_t)((t - t0) / 32) + lane / LPW] = word;
      }
      wave_sync();
      const bool full = !BM && (!PACKED || __ballot(esc));
      if (PACKED && full) {  // rare: ops outside the packed view, from the full columns
        esc_pass<DMAX, GENERAL>(L, nd, u, off0, off1, t0, stride, lane, WAVE, s.incl, a, lr.on ? L.lag_ct : L.pk_vc);
        wave_sync();
      }

      PH(1);
      // ---- 2. records of included ops -> newest birth / kill per group (the next chunk's
      //      loads in flight while one chunk is applied) ----
      for (uint64_t q0 = qa;;) {
        uint64_t q1 = q0 + (uint64_t)VRPT * WAVE;
        if (q1 >= qs && q1 < qe) q1 = qe & ~3ull;  // past the records the zones stood in for
        u32x4 nxt[VRPT / 4];
#pragma unroll
        for (int jj = 0; jj < VRPT / 4; ++jj) {
          const uint64_t q = q1 + (uint64_t)jj * 4 * WAVE + 4 * lane;
          nxt[jj] = q < rk1 ? *(const u32x4 *)(L.rec_g + q) : u32x4{~0u, ~0u, ~0u, ~0u};
        }
#pragma unroll
        for (int jj = 0; jj < VRPT / 4; ++jj) {
          const uint64_t q = q0 + (uint64_t)jj * 4 * WAVE + 4 * lane;
          const uint32_t xs[4] = {rec[jj].x, rec[jj].y, rec[jj].z, rec[jj].w};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const uint32_t x = xs[k];
            if (x == 0xFFFFFFFFu || q + k < rk0 || q + k >= rk1) continue;
            const uint32_t op = AM_REC_OP(x), bit = op + sh;
            if (!((s.incl[bit >> 5] >> (bit & 31)) & 1u)) continue;
            atomicOr(((x & AM_REC_KILL) ? s.killed : s.born) + (AM_REC_GRP(x) >> 5), 1u << (AM_REC_GRP(x) & 31));
            if (by_birth && !(x & AM_REC_KILL)) s.bri[AM_REC_GRP(x)] = (uint16_t)(q + k - rk0);  // a group's one birth
          }
        }
        if (q1 >= rk1) break;
#pragma unroll
        for (int jj = 0; jj < VRPT / 4; ++jj) rec[jj] = nxt[jj];
        q0 = q1;
      }
      wave_sync();
      if (GENERAL) hold(ip);  // the next read's inputs, before this read's stores

      PH(2);
      // ---- 3. scalar outputs (VGPR wave reductions) ----
      uint32_t count = 0, flags = 0, pres = 0;
      uint64_t min_excl = NONE, mxl = 0;
      if (!BM)
        wave_scalars<DMAX, PACKED>(ap, a, full, PACKED ? pk.K : 0, u.allmask, nd, lane, count, flags, pres, min_excl,
                                   mxl);
      int32_t status = (flags & FLAG_BAD) ? AM_ERR_UNEXPECTED_OPERATION : AM_OK;
      const bool ign = u.base_ignore && count == 0;
      const uint32_t opres = ign ? 0u : (pres | u.cpres);
      uint64_t c0 = 0;  // lane d: LastOpCt entry d
#pragma unroll
      for (int d = 0; d < DMAX; ++d)
        if ((uint32_t)d == lane) c0 = u.C0[d];
      const uint64_t myct = (lane < nd && ((opres >> lane) & 1u)) ? umax64(mxl, c0) : 0;

      PH(3);
      // ---- 4. survivors in group order -> the output CSR.  Lane w owns alive word w (G <=
      //      2048 = 64 words): a scan of the popcounts places every survivor, the group ids
      //      are listed in LDS and the pairs gathered 128 at a time, all loads in flight ----
      uint32_t ns = 0;
      const uint32_t nb = uniform_u32(s.slot[j].nb);
      if (nb && status == AM_OK) {
        // 4b. a cached base (vector_orddict snapshot): merge its pairs not killed by an
        //     included candidate with the new survivors (base_merge); a read that outgrows the
        //     LDS lists goes to the next tier untouched
        if (!base_merge<TYPE>(L, B, R, H, s, rk0, G, nb, uniform_u64(s.slot[j].boff), uniform_u64(s.slot[j].ooff),
                              uniform_u32(s.slot[j].ocap), lane, ns, status, by_birth)) {
          if (lane == 0) next.list[atomicAdd(next.count, 1u)] = (uint32_t)r;
          wave_sync();
          continue;
        }
      } else if (status == AM_OK) {
        const uint32_t nwd = (G + 31) / 32;
        const uint32_t aw = lane < nwd ? (s.born[lane] & ~s.killed[lane]) : 0u;
        const uint32_t c = (uint32_t)__popc(aw);
        const uint32_t inc = wave_incl_scan_u32(c, lane);
        ns = (uint32_t)__shfl((int)inc, 63, WAVE);
        uint32_t o = inc - c;
        for (uint32_t bits = aw; bits; bits &= bits - 1) s.list[o++] = (uint16_t)(lane * 32 + __builtin_ctz(bits));
        wave_sync();
        const uint64_t ooff = uniform_u64(s.slot[j].ooff);
        const uint32_t ocap = uniform_u32(s.slot[j].ocap);
        const uint32_t nput = ns < ocap ? ns : ocap;
        for (uint32_t j0 = 0; j0 < nput; j0 += 2 * WAVE) {
          const uint32_t j1 = j0 + lane, j2 = j1 + WAVE;
          u64x2 p1 = {0, 0}, p2 = {0, 0};
          const uint64_t *src = by_birth ? L.prec : L.grp;
          if (j1 < nput) p1 = *(const u64x2 *)(src + 2 * (rk0 + (by_birth ? s.bri[s.list[j1]] : s.list[j1])));
          if (j2 < nput) p2 = *(const u64x2 *)(src + 2 * (rk0 + (by_birth ? s.bri[s.list[j2]] : s.list[j2])));
          if (j1 < nput) R.value.set_a[ooff + j1] = p1.x, R.value.set_b[ooff + j1] = p1.y;
          if (j2 < nput) R.value.set_a[ooff + j2] = p2.x, R.value.set_b[ooff + j2] = p2.y;
          if (j1 < nput) H.put(ooff + j1, p1.x, p1.y, s.list[j1]);
          if (j2 < nput) H.put(ooff + j2, p2.x, p2.y, s.list[j2]);
        }
        if (ns > ocap) status = AM_ERR_CAPACITY;
      }
      PH(4);
      if (BM) {  // the inclusion pass wrote the scalar outputs
        if (lane == 0) {
          if (status == AM_OK) R.value.set_len[r] = ns;
          else R.status[r] = status;
        }
        wave_sync();
        continue;
      }
      if (status == AM_OK && lane < nd) R.last_ct[(uint64_t)lane * B.n_reads + r] = myct;
      if (lane == 0) {
        R.status[r] = status;
        R.flags[r] = (uint8_t)(flags & 0xFFu);
        if (status == AM_OK) {
          R.new_last_op[r] = new_last_op_b(L, s.slot[j].idb, off0, off1, min_excl);
          R.last_ct_ignore[r] = ign ? 1 : 0;
          R.last_ct_pres[r] = opres;
          R.is_new_ss[r] = count > 0;
          R.count[r] = count;
          R.value.set_len[r] = ns;
        }
        if (H.done) H.done[r] = status == AM_OK ? 1 : 0;
      }
      PH(5);
      wave_sync();
    }
    wave_sync();  // the slots are rewritten by the next batch
  }
  if (n_skipped && lane == 0) atomicAdd(H.skipped + AM_STAT_OPS_SKIPPED, (unsigned long long)n_skipped);
  if (n_rskip && lane == 0) atomicAdd(H.skipped + AM_STAT_RECS_SKIPPED, (unsigned long long)n_rskip);
  if (n_gsw && lane == 0) atomicAdd(H.skipped + AM_STAT_GSUM_WORDS, (unsigned long long)n_gsw);
  PH_END();
}

// ---------------------------------------------------------------- split fresh read, pass 1
// A fresh read (the batch clock, no base, no TxId; packed view, no zone index) in two passes:
// k_grp_incl streams the read's commit vectors -- 256-op tiles, one 16-byte load per DC and lane,
// the wave's only live state the tile and the partials -- and writes its inclusion bits into the
// global bitmap ibm (bit p = op slot p) and its scalar outputs {NewLastOp, LastOpCt, IsNewSS,
// Count, status}; k_grp_wave<BM> then streams the records against those bits and gathers the
// survivors.  A wave takes 32 CONSECUTIVE reads at a time and their scalar outputs leave through
// LDS as one coalesced store per column (single-lane stores of reads far apart write partial
// lines of the output columns, each line written back once per writer).
constexpr uint32_t IWB = 32;  // reads per wave batch
__device__ __forceinline__ uint32_t wave_min_u32_v(uint32_t v) {
#define S_(C) v = min(v, dpp32<C>(v));
  AMK_ROW_STEPS(S_)
#undef S_
  v = min(v, (uint32_t)__shfl_xor((int)v, 16, WAVE));
  return min(v, (uint32_t)__shfl_xor((int)v, 32, WAVE));
}
struct ISlot {
  uint64_t off0, K, idb, key;
  uint32_t r, nops;
};
template <int DMAX>
struct ISmem {
  ISlot slot[IWB];
  uint32_t mx[DMAX][WAVE];      // one read's per-lane LastOpCt maxima, transposed for the reduction
  uint64_t ct[DMAX][IWB];       // the batch's outputs, by read
  int64_t nlo[IWB];
  uint32_t count[IWB], pres[IWB];
  int32_t status[IWB];
  uint32_t flags[IWB];
};

// ops [g, g + OPL) of the lane (OPL consecutive slots, g OPL-aligned), packed view: inclusion
// bits (is_op_in_snapshot/7 against the batch clock: every entry X[d] - K <= S[d] - K) and the
// partials.  RANGE: the tile may hold slots outside [off0, off1); escaped ops (x[0] == ESC)
// are left to the caller (esc bit k).
template <int DMAX, int OPL, bool RANGE>
__device__ __forceinline__ uint32_t incl_tile(const uint32_t (&x)[OPL][DMAX], const PkRead<DMAX> &pk, uint64_t g,
                                              uint64_t off0, uint64_t off1, uint32_t (&mx)[DMAX], uint32_t &esc,
                                              uint32_t &cand) {
  uint32_t ib = 0;
#pragma unroll
  for (int k = 0; k < OPL; ++k) {
    const bool e = x[k][0] == AM_PK_ESC;
    const bool inr = !RANGE || (g + k >= off0 && g + k < off1);
    bool in = inr && !e;
#pragma unroll
    for (int d = 0; d < DMAX; ++d) in = in && x[k][d] <= pk.thr[d];
    esc |= (uint32_t)(inr && e) << k;
    cand |= (uint32_t)(inr && !e) << k;
    if (in) {
#pragma unroll
      for (int d = 0; d < DMAX; ++d) mx[d] = max(mx[d], x[k][d]);
    }
    ib |= (uint32_t)in << k;
  }
  return ib;
}

// incl_tile over the lag view: commit entries c (AM_PK_ESC: escaped), four u16 lags per DC in
// lv, the key's lag bases lb; X[d] - K = c - (lb[d] + lag) is rebuilt where it is used (the lags
// stay packed two per register: the rebuilt entries would hold 4 * DMAX registers)
template <int DMAX, bool RANGE>
__device__ __forceinline__ uint32_t incl_tile_lag(const uint32_t (&c)[4], const uint2 (&lv)[DMAX],
                                                  const uint32_t (&lb)[DMAX], const PkRead<DMAX> &pk, uint64_t g,
                                                  uint64_t off0, uint64_t off1, uint32_t (&mx)[DMAX], uint32_t &esc,
                                                  uint32_t &cand) {
  auto xd = [&](int k, int d) -> uint32_t {
    const uint32_t w = k < 2 ? lv[d].x : lv[d].y;
    return c[k] - (lb[d] + ((k & 1) ? w >> 16 : w & 0xFFFFu));
  };
  uint32_t ib = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const bool e = c[k] == AM_PK_ESC;
    const bool inr = !RANGE || (g + k >= off0 && g + k < off1);
    bool in = inr && !e;
#pragma unroll
    for (int d = 0; d < DMAX; ++d) in = in && xd(k, d) <= pk.thr[d];
    esc |= (uint32_t)(inr && e) << k;
    cand |= (uint32_t)(inr && !e) << k;
    if (in) {
#pragma unroll
      for (int d = 0; d < DMAX; ++d) mx[d] = max(mx[d], xd(k, d));
    }
    ib |= (uint32_t)in << k;
  }
  return ib;
}

// LAG: the read streams the lag view (am_op_log.lag_ct / lag / key_lag, 4 + 2 D bytes per op)
// and rebuilds each packed entry X[d] - K = lag_ct - key_lag[d] - lag[d] in u32 (exact: the entry
// fits u32 for every op the view holds); else the packed view (4 D bytes per op)
#ifndef AM_INCL_WAVES
#define AM_INCL_WAVES 3  // waves per SIMD: the pipelined tile loop holds two tiles (168 VGPRs)
#endif
template <int DMAX, int TYPE, bool EXACT, bool LAG>
__global__ void __launch_bounds__(BLOCK, AM_INCL_WAVES) k_grp_incl(am_op_log L, am_read_batch B, am_read_result R, am_sel S,
                                                       am_retry next, uint32_t short_opl, uint32_t *ibm) {
  constexpr int OPL = 4;
  constexpr uint64_t TILE = (uint64_t)WAVE * OPL;
  constexpr uint32_t LPW = 32 / OPL;
  __shared__ ISmem<DMAX> smem[NW];
  ISmem<DMAX> &sm = smem[threadIdx.x >> 6];
  ISlot *sl = sm.slot;
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  const uint64_t lt = (1ull << lane) - 1ull;
  const uint32_t nd = EXACT ? (uint32_t)DMAX : L.n_dc;
  const uint64_t stride = L.snap_stride ? L.snap_stride : L.n_ops;
  const uint32_t sel0 = S.idx ? uniform_u32(S.range[0]) : 0u;
  const uint64_t nsel = S.idx ? (uint64_t)(uniform_u32(S.range[1]) - sel0) : B.n_reads;
  const uint64_t W = (uint64_t)gridDim.x * NW;
  const uint64_t gw = (uint64_t)blockIdx.x * NW + uniform_u32(threadIdx.x >> 6);
  const uint64_t n = B.n_reads;
  ReadU<DMAX> u;
  read_inputs<DMAX, false, true>(L, nd, B, 0, u);  // one clock, no bases / TxIds

  for (uint64_t b0 = gw * IWB; b0 < nsel; b0 += (uint64_t)IWB * W) {
    // ---- lane j < IWB: read b0 + j -> slot j (errors and hand-offs leave here) ----
    const uint64_t ii = b0 + lane;
    bool elig = false, hand = false;
    uint64_t rr = 0;
    if (lane < IWB && ii < nsel) {
      GMeta mm;
      read_meta(L, B, S.idx ? (uint64_t)S.idx[sel0 + ii] : ii, TYPE, mm);
      rr = mm.r;
      if (mm.st != AM_OK) {
        R.status[mm.r] = mm.st, R.flags[mm.r] = 0;
      } else if (!wave_takes(L, B, mm, short_opl)) {
        hand = true;
      } else {
        elig = true;
        ISlot &w = sl[lane];
        w.off0 = mm.off0, w.K = L.key_tbase[mm.key], w.idb = L.key_id_base ? L.key_id_base[mm.key] : 1;
        w.key = mm.key;
        w.r = (uint32_t)mm.r, w.nops = (uint32_t)(mm.off1 - mm.off0);
      }
    }
    const uint64_t hm = __ballot(hand);
    if (hm) {
      uint32_t base = 0;
      if (lane == 0) base = atomicAdd(next.count, (uint32_t)__popcll(hm));
      base = uniform_u32(base);
      if (hand) next.list[base + (uint32_t)__popcll(hm & lt)] = (uint32_t)rr;
    }
    const uint64_t emask = __ballot(elig);
    wave_sync();

    for (uint64_t em = emask; em; em &= em - 1) {
      const uint32_t j = (uint32_t)__builtin_ctzll(em);
      const uint64_t off0 = uniform_u64(sl[j].off0), off1 = off0 + uniform_u32(sl[j].nops);
      PkRead<DMAX> pk;
      pk_setup(u, nd, uniform_u64(sl[j].K), pk);
      uint32_t mx[DMAX], lb[DMAX];  // lb: the key's lag bases (LAG)
#pragma unroll
      for (int d = 0; d < DMAX; ++d) mx[d] = 0;
      if (LAG) {
        const uint64_t key = uniform_u64(sl[j].key);
#pragma unroll
        for (int d = 0; d < DMAX; ++d) lb[d] = uniform_u32(d < (int)nd ? (uint32_t)L.key_lag[key * nd + d] : 0u);
      }
      uint32_t cnt = 0, minex = 0xFFFFFFFFu, anyc = 0, anyesc = 0;
      uint64_t escm = 0;  // the lane's escaped ops: bit OPL * tile + k (the first 64 / OPL tiles)
      const uint64_t t0 = off0 & ~31ull;  // 32-op aligned: lane groups of LPW fill whole bitmap words
      // one tile's inclusion bits -> partials, escape marks and the bitmap words
      auto tile_out = [&](uint64_t t, uint64_t g, uint32_t ib, uint32_t esc, uint32_t cand) {
        if (pk.never) ib = 0;
        cnt += (uint32_t)__popc(ib);
        anyc |= cand;
        anyesc |= esc;
        const uint64_t ti = (t - t0) / TILE;
        if (esc) escm |= ti < 64 / OPL ? (uint64_t)esc << (OPL * ti) : ~0ull;  // ~0: walk the key
        const uint32_t ex = cand & ~ib;
        if (ex) minex = min(minex, (uint32_t)(g - t0) + (uint32_t)__builtin_ctz(ex));
        uint32_t word = ib << (OPL * (lane % LPW));
#pragma unroll
        for (uint32_t xo = 1; xo < LPW; xo <<= 1) word |= (uint32_t)__shfl_xor((int)word, (int)xo);
        const uint64_t w0 = g & ~31ull;  // this lane group's word: ops [w0, w0 + 32)
        if (lane % LPW == 0 && w0 < off1) {
          if (w0 >= off0 && w0 + 32 <= off1) {
            ibm[w0 >> 5] = word;
          } else {  // a word shared with a neighbouring key: only this read's bits change
            const uint32_t lo = off0 > w0 ? (uint32_t)(off0 - w0) : 0u;
            const uint32_t hi = off1 < w0 + 32 ? (uint32_t)(off1 - w0) : 32u;
            const uint32_t mask = (hi >= 32 ? ~0u : ((1u << hi) - 1u)) & ~((1u << lo) - 1u);
            atomicAnd(ibm + (w0 >> 5), ~mask);
            atomicOr(ibm + (w0 >> 5), word & mask);
          }
        }
      };
      if constexpr (LAG) {
        static_assert(OPL == 4, "four u16 lags per 8-byte load");
        // software-pipelined: tile t + 1's loads are issued before tile t is evaluated, into the
        // other of two register sets (no copies between them: a copy would wait for the loads)
        uint32_t cA[OPL], cB[OPL];
        uint2 lA[DMAX], lB[DMAX];
        auto load = [&](uint64_t t, uint32_t (&c)[OPL], uint2 (&lv)[DMAX]) {
          const uint64_t g = t + (uint64_t)lane * OPL;
#pragma unroll
          for (int k = 0; k < OPL; ++k) c[k] = 0;
          if (g < off1) ld_n32<OPL>(L.lag_ct + g, c);
#pragma unroll
          for (int d = 0; d < DMAX; ++d) {
            lv[d] = uint2{0, 0};
            if (d < (int)nd && g < off1) lv[d] = *(const uint2 *)(L.lag + (uint64_t)d * stride + g);
          }
        };
        auto eval = [&](uint64_t t, const uint32_t (&c)[OPL], const uint2 (&lv)[DMAX]) {
          const uint64_t g = t + (uint64_t)lane * OPL;
          uint32_t esc = 0, cand = 0;
          const bool whole = t >= off0 && t + TILE <= off1;
          // (pad DCs d >= nd: c - lb[d] with lb = 0 lies under the always-passing pad threshold)
          const uint32_t ib = whole ? incl_tile_lag<DMAX, false>(c, lv, lb, pk, g, off0, off1, mx, esc, cand)
                                    : incl_tile_lag<DMAX, true>(c, lv, lb, pk, g, off0, off1, mx, esc, cand);
          tile_out(t, g, ib, esc, cand);
        };
        load(t0, cA, lA);
        for (uint64_t t = t0; t < off1; t += 2 * TILE) {
          const uint64_t t1 = t + TILE;
          if (t1 < off1) load(t1, cB, lB);
          eval(t, cA, lA);
          if (t1 >= off1) break;
          if (t1 + TILE < off1) load(t1 + TILE, cA, lA);
          eval(t1, cB, lB);
        }
      } else {
        for (uint64_t t = t0; t < off1; t += TILE) {
          const uint64_t g = t + (uint64_t)lane * OPL;
          uint32_t esc = 0, cand = 0;
          const bool whole = t >= off0 && t + TILE <= off1;
          uint32_t x[OPL][DMAX];
#pragma unroll
          for (int d = 0; d < DMAX; ++d) {
            uint32_t q[OPL] = {};
            if (d < (int)nd && g < off1) ld_n32<OPL>(L.pk_vc + (uint64_t)d * stride + g, q);
#pragma unroll
            for (int k = 0; k < OPL; ++k) x[k][d] = q[k];
          }
          const uint32_t ib = whole ? incl_tile<DMAX, OPL, false>(x, pk, g, off0, off1, mx, esc, cand)
                                    : incl_tile<DMAX, OPL, true>(x, pk, g, off0, off1, mx, esc, cand);
          tile_out(t, g, ib, esc, cand);
        }
      }
      // ---- the read's scalar outputs: LastOpCt maxima reduced through LDS (lane 8 d + c takes
      //      DC d's entries of lanes 8 c .. 8 c + 7, then an 8-lane max), the rest by DPP ----
#pragma unroll
      for (int d = 0; d < DMAX; ++d) sm.mx[d][lane] = mx[d];
      const uint32_t count_p = wave_sum_u32_v(cnt);
      minex = wave_min_u32_v(minex);
      const bool cands = __ballot(anyc != 0) != 0;
      const bool escs = __ballot(anyesc != 0) != 0;
      wave_sync();
      uint32_t m = 0;
      {
        const uint32_t d = lane >> 3, c = lane & 7u;
        if (d < (uint32_t)DMAX) {
          const u32x4 a0 = *(const u32x4 *)&sm.mx[d][8 * c], a1 = *(const u32x4 *)&sm.mx[d][8 * c + 4];
          m = max(max(max(a0.x, a0.y), max(a0.z, a0.w)), max(max(a1.x, a1.y), max(a1.z, a1.w)));
        }
        m = max(m, (uint32_t)__shfl_xor((int)m, 1));
        m = max(m, (uint32_t)__shfl_xor((int)m, 2));
        m = max(m, (uint32_t)__shfl_xor((int)m, 4));
      }
      // lane d: DC d's packed maximum (relative to K)
      const uint32_t mxd = (uint32_t)__shfl((int)m, (int)((lane & 7u) << 3));
      uint64_t mxl = (lane < nd && count_p) ? pk.K + mxd : 0;
      uint32_t count = count_p, flags = cands ? pk.miss : 0u, pres = count_p ? u.allmask : 0u;
      uint64_t min_excl = minex == 0xFFFFFFFFu ? NONE : t0 + minex;
      if (escs) {  // rare: ops outside the packed view, from the full columns (bits ORed in)
        Acc<DMAX> a;
        a.reset();
        __builtin_amdgcn_s_waitcnt(0);
        if (__ballot(escm == ~0ull)) {  // a long key's late tiles: the wave walks its escape marks
          esc_pass_g<DMAX>(L, nd, u, off0, off1, stride, lane, ibm, a, LAG ? L.lag_ct : L.pk_vc);
        } else {  // the lane's own escaped ops, marked by the tile loop: no second walk of the key
          for (uint64_t m = escm; m; m &= m - 1) {
            const uint32_t b = (uint32_t)__builtin_ctzll(m);
            const uint64_t p = t0 + (uint64_t)(b / OPL) * TILE + (uint64_t)lane * OPL + b % OPL;
            uint64_t sv[DMAX], ct;
            uint32_t meta;
            esc_load<DMAX>(L, nd, stride, p, sv, ct, meta);
            if (eval_op<DMAX, false>(u, meta, ct, sv, u.allmask, false, p, a) && !(meta & AM_META_BAD))
              atomicOr(&ibm[p >> 5], 1u << (p & 31));
          }
        }
        count += wave_sum_u32_v(a.count), flags |= wave_or_u32_v(a.flags), pres |= wave_or_u32_v(a.pres);
        min_excl = wave_min_u64_v(umin64(min_excl, a.min_excl));
#pragma unroll
        for (int d = 0; d < DMAX; ++d) {
          if (d >= (int)nd) continue;
          const uint64_t am = wave_max_u64_v(a.mx[d]);
          if ((uint32_t)d == lane) mxl = umax64(mxl, am);
        }
      }
      // the read's outputs into the batch's LDS rows (slot j); they leave with the batch
      const bool ign = count == 0;  // base ignore
      const uint32_t opres = ign ? 0u : pres;
      if (lane < nd) sm.ct[lane][j] = ((opres >> lane) & 1u) ? mxl : 0;
      if (lane == 0) {
        sm.status[j] = (flags & FLAG_BAD) ? AM_ERR_UNEXPECTED_OPERATION : AM_OK;
        sm.flags[j] = flags & 0xFFu;
        sm.count[j] = count;
        sm.pres[j] = opres;
        sm.nlo[j] = new_last_op_b(L, uniform_u64(sl[j].idb), off0, off1, min_excl);
      }
      wave_sync();  // sm.mx is rewritten by the next read
    }
    // ---- the batch's outputs: one coalesced store per column (lane j: read b0 + j) ----
    if ((emask >> lane) & 1ull) {
      const uint64_t r = rr;
      const int32_t st = sm.status[lane];
      R.status[r] = st;
      R.flags[r] = (uint8_t)sm.flags[lane];
      if (st == AM_OK) {
        const uint32_t c = sm.count[lane];
        R.new_last_op[r] = sm.nlo[lane];
        R.last_ct_ignore[r] = c == 0 ? 1 : 0;
        R.last_ct_pres[r] = sm.pres[lane];
        R.is_new_ss[r] = c > 0;
        R.count[r] = c;
#pragma unroll
        for (int d = 0; d < DMAX; ++d)
          if (d < (int)nd) R.last_ct[(uint64_t)d * n + r] = sm.ct[d][lane];
      }
    }
    wave_sync();  // the slots are rewritten by the next batch
  }
}

// ---------------------------------------------------------------- split fresh read, pass 2
// k_grp_recs: the records of the reads k_grp_incl took, against its bitmap, and the survivors'
// pairs.  Latency-bound (a read is a few KB), so a wave keeps the NEXT read's bitmap words and
// first two record chunks in flight while it applies this read's records and gathers its
// survivors; LDS per wave is a few KB (survivor list in rounds), so ~5 waves per SIMD.
constexpr uint32_t RCH = 512;    // records per chunk: two 16-byte loads per lane
constexpr uint32_t RLIST = 256;  // survivor-list entries per gather round
struct RSlot {
  uint64_t off0, rk0, ooff;
  uint32_t r, nops, nrec, G, ocap, ok;
};
struct RSmem {
  uint32_t born[VG / 32], killed[VG / 32];
  uint32_t incl[VWORDS];
  uint16_t list[RLIST];
  uint16_t bri[VG];  // per group: its birth record (from the read's rk0), set with its born bit
  RSlot slot[IWB];
};
struct RPre {  // a read's prefetched inputs: one bitmap word and two record chunks per lane
  uint32_t w;
  u32x4 c[4];
};

template <int DMAX, int TYPE>
__global__ void __launch_bounds__(BLOCK, 5) k_grp_recs(am_op_log L, am_read_batch B, am_read_result R, am_sel S,
                                                       uint32_t short_opl, const uint32_t *ibm) {
  __shared__ RSmem smem[NW];
  RSmem &s = smem[threadIdx.x >> 6];
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  const uint32_t sel0 = S.idx ? uniform_u32(S.range[0]) : 0u;
  const uint64_t nsel = S.idx ? (uint64_t)(uniform_u32(S.range[1]) - sel0) : B.n_reads;
  const uint64_t W = (uint64_t)gridDim.x * NW;
  const uint64_t gw = (uint64_t)blockIdx.x * NW + uniform_u32(threadIdx.x >> 6);
  const uint64_t *const pairs = L.prec ? L.prec : L.grp;

  // prefetch read j of the slot table: bitmap words [t0 / 32, ...) (lane i: word i, the first
  // 64), records [rk0 & ~3, + 2 RCH)
  auto pre = [&](uint32_t j, RPre &p) {
    const uint64_t off0 = s.slot[j].off0, rk0 = s.slot[j].rk0;
    const uint32_t nops = s.slot[j].nops, nrec = s.slot[j].nrec;
    const uint64_t t0 = off0 & ~31ull, rk1 = rk0 + nrec;
    const uint32_t nw = (uint32_t)((off0 + nops - t0 + 31) / 32);
    p.w = lane < nw ? ibm[(t0 >> 5) + lane] : 0u;
    const uint64_t qa = rk0 & ~3ull;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const uint64_t q = qa + (uint64_t)c * 4 * WAVE + 4 * lane;
      p.c[c] = q < rk1 ? *(const u32x4 *)(L.rec_g + q) : u32x4{~0u, ~0u, ~0u, ~0u};
    }
  };
  // records [q, q + 4) against the LDS bitmap (bit = op + sh) -> born / killed bits
  auto apply4 = [&](u32x4 v, uint64_t q, uint64_t rk0, uint64_t rk1, uint32_t sh) {
    const uint32_t xs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t x = xs[k];
      if (x == 0xFFFFFFFFu || q + k < rk0 || q + k >= rk1) continue;
      const uint32_t bit = AM_REC_OP(x) + sh;
      if (!((s.incl[bit >> 5] >> (bit & 31)) & 1u)) continue;
      const uint32_t g = AM_REC_GRP(x);
      atomicOr(((x & AM_REC_KILL) ? s.killed : s.born) + (g >> 5), 1u << (g & 31));
      if (!(x & AM_REC_KILL)) s.bri[g] = (uint16_t)(q + k - rk0);  // a group's one birth
    }
  };

  for (uint64_t b0 = gw * IWB; b0 < nsel; b0 += (uint64_t)IWB * W) {
    // ---- lane j < IWB: read b0 + j -> slot j (the reads k_grp_incl took and left ok) ----
    const uint64_t ii = b0 + lane;
    bool ok = false;
    if (lane < IWB && ii < nsel) {
      GMeta mm;
      read_meta(L, B, S.idx ? (uint64_t)S.idx[sel0 + ii] : ii, TYPE, mm);
      ok = mm.st == AM_OK && wave_takes(L, B, mm, short_opl) && R.status[mm.r] == AM_OK;
      if (ok) {
        RSlot &w = s.slot[lane];
        const uint64_t o0 = R.value.set_off[mm.r], o1 = R.value.set_off[mm.r + 1];
        w.off0 = mm.off0, w.rk0 = mm.rk0, w.ooff = o0;
        w.r = (uint32_t)mm.r, w.nops = (uint32_t)(mm.off1 - mm.off0), w.nrec = (uint32_t)(mm.rk1 - mm.rk0);
        w.G = mm.G, w.ocap = o1 - o0 < 0xFFFFFFFFull ? (uint32_t)(o1 - o0) : 0xFFFFFFFFu;
      }
    }
    uint64_t em = __ballot(ok);
    wave_sync();
    RPre cur;
    if (em) pre((uint32_t)__builtin_ctzll(em), cur);
    uint32_t setlen = 0;  // lane j: read j's survivor count
    int32_t cap_err = 0;  // lane j: read j overflowed its capacity
    for (; em; em &= em - 1) {
      const uint32_t j = (uint32_t)__builtin_ctzll(em);
      const uint64_t off0 = uniform_u64(s.slot[j].off0), rk0 = uniform_u64(s.slot[j].rk0);
      const uint64_t off1 = off0 + uniform_u32(s.slot[j].nops), rk1 = rk0 + uniform_u32(s.slot[j].nrec);
      const uint32_t G = uniform_u32(s.slot[j].G);
      const uint64_t t0 = off0 & ~31ull;
      const uint32_t sh = (uint32_t)(off0 - t0), nw = (uint32_t)((off1 - t0 + 31) / 32);
      // this read's bitmap into LDS (words past the first 64 straight from memory: long logs)
      if (lane < nw) s.incl[lane] = cur.w;
      for (uint32_t i = WAVE + lane; i < nw; i += WAVE) s.incl[i] = ibm[(t0 >> 5) + i];
      for (uint32_t g = lane; g < (G + 31) / 32; g += WAVE) s.born[g] = 0, s.killed[g] = 0;
      u32x4 c[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) c[k] = cur.c[k];
      // the next read's inputs in flight from here on
      const uint64_t rest = em & (em - 1);
      if (rest) pre((uint32_t)__builtin_ctzll(rest), cur);
      wave_sync();
      // ---- records: the two prefetched chunks, then the rest two chunks at a time ----
      const uint64_t qa = rk0 & ~3ull;
#pragma unroll
      for (int k = 0; k < 4; ++k) apply4(c[k], qa + (uint64_t)k * 4 * WAVE + 4 * lane, rk0, rk1, sh);
      for (uint64_t q0 = qa + 2 * RCH; q0 < rk1; q0 += 2 * RCH) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint64_t q = q0 + (uint64_t)k * 4 * WAVE + 4 * lane;
          c[k] = q < rk1 ? *(const u32x4 *)(L.rec_g + q) : u32x4{~0u, ~0u, ~0u, ~0u};
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) apply4(c[k], q0 + (uint64_t)k * 4 * WAVE + 4 * lane, rk0, rk1, sh);
      }
      wave_sync();
      // ---- survivors in group order: lane w owns alive word w; listed in rounds of RLIST ----
      const uint32_t nwd = (G + 31) / 32;
      const uint32_t aw = lane < nwd ? (s.born[lane] & ~s.killed[lane]) : 0u;
      const uint32_t cnt = (uint32_t)__popc(aw);
      const uint32_t inc = wave_incl_scan_u32(cnt, lane);
      const uint32_t ns = (uint32_t)__shfl((int)inc, 63, WAVE);
      const uint64_t ooff = uniform_u64(s.slot[j].ooff);
      const uint32_t ocap = uniform_u32(s.slot[j].ocap);
      const uint32_t nput = ns < ocap ? ns : ocap;
      for (uint32_t base = 0; base < nput; base += RLIST) {
        uint32_t o = inc - cnt;
        for (uint32_t bits = aw; bits; bits &= bits - 1, ++o)
          if (o >= base && o < base + RLIST) s.list[o - base] = (uint16_t)(lane * 32 + __builtin_ctz(bits));
        wave_sync();
        const uint32_t end = nput - base < RLIST ? nput - base : RLIST;
        for (uint32_t j0 = 0; j0 < end; j0 += 2 * WAVE) {
          const uint32_t j1 = j0 + lane, j2 = j1 + WAVE;
          u64x2 p1 = {0, 0}, p2 = {0, 0};
          // a survivor's pair through its birth record (prec: births close together in op
          // order) rather than its group slot (grp: one group run apart in output order)
          if (j1 < end) p1 = *(const u64x2 *)(pairs + 2 * (rk0 + (L.prec ? s.bri[s.list[j1]] : s.list[j1])));
          if (j2 < end) p2 = *(const u64x2 *)(pairs + 2 * (rk0 + (L.prec ? s.bri[s.list[j2]] : s.list[j2])));
          if (j1 < end) R.value.set_a[ooff + base + j1] = p1.x, R.value.set_b[ooff + base + j1] = p1.y;
          if (j2 < end) R.value.set_a[ooff + base + j2] = p2.x, R.value.set_b[ooff + base + j2] = p2.y;
        }
        wave_sync();
      }
      if (lane == j) setlen = ns, cap_err = ns > ocap;
      wave_sync();
    }
    // ---- the batch's outputs (lane j: read b0 + j): set_len, or the capacity status ----
    if (ok) {
      const uint64_t r = s.slot[lane].r;
      if (cap_err) R.status[r] = AM_ERR_CAPACITY;
      else R.value.set_len[r] = setlen;
    }
    wave_sync();  // the slots are rewritten by the next batch
  }
}

// ---------------------------------------------------------------- 16-lane row per short read
// A wave takes 64 reads at a time: lane i checks read i against the row limits (the others
// leave through one hand-off atomic per wave), then the four 16-lane rows walk the
// eligible reads, one read per row per step: op sl + 16k, records sl + 16j, groups sl + 16j.
constexpr uint32_t ROW_OPS = 64, ROW_REC = 128, ROW_G = 64;
constexpr int RG = 16;

struct RowGSmem {
  uint32_t born[ROW_G / 32], killed[ROW_G / 32];
};

template <int DMAX, int TYPE, bool GENERAL, bool PACKED, bool EXACT>
__global__ void __launch_bounds__(BLOCK) k_grp_row(am_op_log L, am_read_batch B, am_read_result R, am_sel S,
                                                   am_retry next) {
  __shared__ RowGSmem rsm[BLOCK / RG];
  RowGSmem &s = rsm[threadIdx.x / RG];
  const uint32_t lane = threadIdx.x & (WAVE - 1), row = lane / RG, sl = lane % RG;
  const uint64_t lt = (1ull << lane) - 1ull;
  const uint32_t nd = EXACT ? (uint32_t)DMAX : L.n_dc;  // EXACT: n_dc == DMAX, no per-DC guards
  const uint64_t stride = L.snap_stride ? L.snap_stride : L.n_ops;
  const uint32_t sel0 = S.idx ? uniform_u32(S.range[0]) : 0u;
  const uint64_t nsel = S.idx ? (uint64_t)(uniform_u32(S.range[1]) - sel0) : B.n_reads;
  const uint64_t W = (uint64_t)gridDim.x * (BLOCK / WAVE);
  const uint64_t gw = (uint64_t)blockIdx.x * (BLOCK / WAVE) + uniform_u32(threadIdx.x >> 6);
  const uint64_t n_batches = (nsel + WAVE - 1) / WAVE;

  for (uint64_t bid = gw; bid < n_batches; bid += W) {
    // ---- lane i: read rb + i, checked against the row limits ----
    const uint64_t rb = bid * WAVE;
    const uint32_t nb = (uint32_t)(nsel - rb < (uint64_t)WAVE ? nsel - rb : (uint64_t)WAVE);
    GMeta mi;
    mi.st = AM_OK, mi.G = AM_NGRP_NONE, mi.off0 = mi.off1 = mi.rk0 = mi.rk1 = 0, mi.key = 0, mi.r = 0;
    if (lane < nb) read_meta(L, B, S.idx ? (uint64_t)S.idx[sel0 + rb + lane] : rb + lane, TYPE, mi);
    const bool ok_i = lane < nb && mi.st == AM_OK && mi.G != AM_NGRP_NONE && mi.off1 - mi.off0 <= ROW_OPS &&
                      mi.rk1 - mi.rk0 <= ROW_REC && mi.G <= ROW_G && !has_base_pairs(B, mi.r);
    if (lane < nb && mi.st != AM_OK) R.status[mi.r] = mi.st, R.flags[mi.r] = 0;
    const uint64_t hm = __ballot(lane < nb && mi.st == AM_OK && !ok_i);
    if (hm) {
      uint32_t base = 0;
      if (lane == 0) base = atomicAdd(next.count, (uint32_t)__popcll(hm));
      base = uniform_u32(base);
      if ((hm >> lane) & 1ull) next.list[base + (uint32_t)__popcll(hm & lt)] = (uint32_t)mi.r;
    }
    uint64_t emask = __ballot(ok_i);
    while (emask) {
      // row q takes the q-th eligible read left in the batch
      uint64_t mm = emask;
      for (uint32_t q = 0; q < row && mm; ++q) mm &= mm - 1;
      const bool ok = mm != 0;
      const uint32_t j = ok ? (uint32_t)__builtin_ctzll(mm) : 0u;
      for (uint32_t q = 0; q < 4 && emask; ++q) emask &= emask - 1;
      GMeta m;
      m.r = shfl_u64(mi.r, j), m.key = shfl_u64(mi.key, j);
      m.off0 = shfl_u64(mi.off0, j), m.off1 = shfl_u64(mi.off1, j);
      m.rk0 = shfl_u64(mi.rk0, j), m.rk1 = shfl_u64(mi.rk1, j);
      m.G = shfl_u32(mi.G, j), m.st = AM_OK;
      ReadU<DMAX> u;
      if (ok) {
        read_inputs<DMAX, GENERAL, false>(L, nd, B, m.r, u);
      } else {
        u.allmask = 0, u.spres = 0, u.cpres = 0, u.base_ignore = true, u.has_txid = false, u.txid = 0;
#pragma unroll
        for (int d = 0; d < DMAX; ++d) u.S[d] = 0, u.C0[d] = 0;
      }
      if (sl < ROW_G / 32) s.born[sl] = 0, s.killed[sl] = 0;
      // the read's records (one per lane and step), in flight with the ops
      uint32_t rec[ROW_REC / RG];
#pragma unroll
      for (uint32_t k = 0; k < ROW_REC / RG; ++k) {
        const uint64_t q = m.rk0 + sl + RG * k;
        rec[k] = (ok && q < m.rk1) ? L.rec_g[q] : 0xFFFFFFFFu;
      }
      // ---- ops: op sl + 16k of the read ----
      PkRead<DMAX> pk;
      if (PACKED) pk_setup(u, nd, ok ? L.key_tbase[m.key] : 0, pk);
      Acc<DMAX> a;
      AccP<DMAX> ap;
      a.reset();
      ap.reset();
      bool esc = false;
      uint64_t incl = 0;
      // one op from the full columns (full view, or an op outside the packed view)
      auto eval_full = [&](uint64_t p) -> bool {
        uint64_t svf[DMAX], ct;
        uint32_t meta;
        esc_load<DMAX>(L, nd, stride, p, svf, ct, meta);  // (the columns when the op has no row)
        const uint32_t sp = (GENERAL && L.snap_pres) ? L.snap_pres[p] : u.allmask;
        const bool txm = GENERAL && u.has_txid && L.op_txid[p] == u.txid;
        return eval_op<DMAX, GENERAL>(u, meta, ct, svf, sp, txm, p, a) && !(meta & AM_META_BAD);
      };
#pragma unroll
      for (uint32_t k = 0; k < ROW_OPS / RG; ++k) {
        const uint64_t p = m.off0 + sl + RG * k;
        bool in = false;
        if (ok && p < m.off1) {
          if (PACKED) {
            uint32_t x[DMAX];
#pragma unroll
            for (int d = 0; d < DMAX; ++d) x[d] = d < (int)nd ? L.pk_vc[(uint64_t)d * stride + p] : 0u;
            const bool txm = GENERAL && u.has_txid && L.op_txid[p] == u.txid;
            if (x[0] == AM_PK_ESC) esc = true;
            else in = pk_eval<DMAX, GENERAL>(pk, u, x, txm, p, ap);
          } else {
            in = eval_full(p);
          }
        }
        incl |= ((__ballot(in) >> (row * RG)) & 0xFFFFull) << (RG * k);
      }
      if (PACKED && __ballot(esc)) {  // rare: ops outside the packed view, from the full columns
#pragma unroll
        for (uint32_t k = 0; k < ROW_OPS / RG; ++k) {
          const uint64_t p = m.off0 + sl + RG * k;
          const bool in = ok && p < m.off1 && L.pk_vc[p] == AM_PK_ESC && eval_full(p);
          incl |= ((__ballot(in) >> (row * RG)) & 0xFFFFull) << (RG * k);
        }
      }
      wave_sync();
      // ---- records of included ops -> newest birth / kill per group ----
#pragma unroll
      for (uint32_t k = 0; k < ROW_REC / RG; ++k) {
        const uint32_t x = rec[k];
        if (x == 0xFFFFFFFFu) continue;
        const uint32_t op = AM_REC_OP(x);
        if (!((incl >> op) & 1ull)) continue;
        atomicOr(((x & AM_REC_KILL) ? s.killed : s.born) + (AM_REC_GRP(x) >> 5), 1u << (AM_REC_GRP(x) & 31));
      }
      wave_sync();
      // ---- scalar outputs: row reductions (full EXEC) ----
      if (PACKED) pk_fold(ap, pk.K, u.allmask, a);
      const uint32_t count = row_sum_u32(a.count), flags = row_or_u32(a.flags), pres = row_or_u32(a.pres);
      const uint64_t min_excl = row_min_u64(a.min_excl);
      uint64_t mx[DMAX];
#pragma unroll
      for (int d = 0; d < DMAX; ++d) mx[d] = d < (int)nd ? row_max_u64(a.mx[d]) : 0;
      int32_t status = (flags & FLAG_BAD) ? AM_ERR_UNEXPECTED_OPERATION : AM_OK;
      // ---- survivors in group order ----
      uint32_t ns = 0;
      const uint64_t ooff = ok ? R.value.set_off[m.r] : 0, ocap = ok ? R.value.set_off[m.r + 1] - ooff : 0;
#pragma unroll
      for (uint32_t k = 0; k < ROW_G / RG; ++k) {
        const uint32_t g = sl + RG * k;
        const bool alive =
            ok && status == AM_OK && g < m.G && (((s.born[g >> 5] & ~s.killed[g >> 5]) >> (g & 31)) & 1u);
        const uint32_t rm = (uint32_t)((__ballot(alive) >> (row * RG)) & 0xFFFFu);
        if (alive) {
          const uint64_t o = ns + (uint32_t)__popc(rm & ((1u << sl) - 1u));
          if (o < ocap) {
            const u64x2 ab = *(const u64x2 *)(L.grp + 2 * (m.rk0 + g));
            R.value.set_a[ooff + o] = ab.x;
            R.value.set_b[ooff + o] = ab.y;
          }
        }
        ns += (uint32_t)__popc(rm);
      }
      if (ok && status == AM_OK && ns > ocap) status = AM_ERR_CAPACITY;
      if (ok && sl == 0) write_scalars<DMAX>(L, nd, B, R, m, u, status, count, flags, pres, min_excl, mx, ns);
      wave_sync();
    }
  }
}

// ---------------------------------------------------------------- launchers
// the split fresh read: k_grp_incl (op stream -> inclusion bitmap + scalars), then the record /
// survivor pass k_grp_recs
template <int D, int TYPE, bool EXACT>
int launch_split(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S,
                 am_retry next, uint32_t short_opl) {
  const uint64_t stride = L->snap_stride ? L->snap_stride : L->n_ops;
  void *ibm = nullptr;
  if (int rc = am_ctx_scratch(ctx, AM_SCR_INCL, (stride / 32 + 4) * 4, &ibm)) return rc;
  // the lag view when the log has it: 4 + 2 D bytes of commit vector per op instead of 4 D
  const bool lag = L->lag_ct && L->lag && L->key_lag;
  static int occ_i = 0, occ_w = 0;
  if (!occ_i) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ_i, k_grp_incl<D, TYPE, EXACT, true>, BLOCK, 0) !=
            hipSuccess ||
        occ_i < 1)
      occ_i = 2;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ_w, k_grp_recs<D, TYPE>, BLOCK, 0) != hipSuccess ||
        occ_w < 1)
      occ_w = 1;
  }
  const uint64_t want_i = (B->n_reads + NW * IWB - 1) / (NW * IWB), want_w = want_i;
  const uint64_t bi = want_i < (uint64_t)ctx->n_cu * occ_i ? want_i : (uint64_t)ctx->n_cu * occ_i;
  const uint64_t bw = want_w < (uint64_t)ctx->n_cu * occ_w ? want_w : (uint64_t)ctx->n_cu * occ_w;
  if (bi == 0) return AM_OK;
  if (lag)
    hipLaunchKernelGGL((k_grp_incl<D, TYPE, EXACT, true>), dim3((unsigned)bi), dim3(BLOCK), 0, ctx->stream, *L, *B, *R,
                       S, next, short_opl, (uint32_t *)ibm);
  else
    hipLaunchKernelGGL((k_grp_incl<D, TYPE, EXACT, false>), dim3((unsigned)bi), dim3(BLOCK), 0, ctx->stream, *L, *B,
                       *R, S, next, short_opl, (uint32_t *)ibm);
  hipLaunchKernelGGL((k_grp_recs<D, TYPE>), dim3((unsigned)bw), dim3(BLOCK), 0, ctx->stream, *L, *B, *R, S,
                     short_opl, (const uint32_t *)ibm);
  AM_HIP(hipGetLastError());
  return AM_OK;
}

template <int D, int TYPE, bool GENERAL, bool PACKED, bool EXACT>
int launch_d(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S, am_retry next,
             int tier) {
  if ((tier & 0xFF) == AM_GRP_WAVE) {
    const uint32_t short_opl = (tier & AM_GRP_HAND_SHORT) ? (D <= 8 ? 8u : 4u) : 0u;  // am_lanes.hip lopl
    constexpr size_t smem = sizeof(WaveSmem) * NW;
    if constexpr (!GENERAL && PACKED && D <= 8) {
      if (!L->zone_vc && !ctx->tee_a) return launch_split<D, TYPE, EXACT>(ctx, L, B, R, S, next, short_opl);
    }
    static int occ = 0;
    if (!occ) {
      AM_HIP(hipFuncSetAttribute((const void *)k_grp_wave<D, TYPE, GENERAL, PACKED, EXACT>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_grp_wave<D, TYPE, GENERAL, PACKED, EXACT>, BLOCK,
                                                       smem) != hipSuccess || occ < 1)
        occ = 1;
    }
    uint64_t blocks = (B->n_reads + NW - 1) / NW, cap = (uint64_t)ctx->n_cu * occ;
    if (blocks > cap) blocks = cap;
    if (blocks == 0) return AM_OK;
    hipLaunchKernelGGL((k_grp_wave<D, TYPE, GENERAL, PACKED, EXACT>), dim3((unsigned)blocks), dim3(BLOCK), smem,
                       ctx->stream, *L, *B, *R, S, next, short_opl, GrpHint{ctx->grp_hint_in, ctx->tee_a, ctx->tee_b, ctx->tee_g, ctx->tee_shift,
                                                                  ctx->tee_done,
                                                                  (unsigned long long *)ctx->stats});
  } else if (tier == AM_GRP_ROW) {
    static int occ = 0;
    if (!occ) {
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_grp_row<D, TYPE, GENERAL, PACKED, EXACT>, BLOCK, 0) !=
              hipSuccess || occ < 1)
        occ = 2;
    }
    const uint64_t waves = (B->n_reads + WAVE - 1) / WAVE;
    uint64_t blocks = (waves + NW - 1) / NW, cap = (uint64_t)ctx->n_cu * occ;
    if (blocks > cap) blocks = cap;
    if (blocks == 0) return AM_OK;
    hipLaunchKernelGGL((k_grp_row<D, TYPE, GENERAL, PACKED, EXACT>), dim3((unsigned)blocks), dim3(BLOCK), 0,
                       ctx->stream, *L, *B, *R, S, next);
  } else {
    constexpr size_t smem = sizeof(WgSmem<D>);
    static int occ = 0;
    if (!occ) {
      AM_HIP(hipFuncSetAttribute((const void *)k_grp_wg<D, TYPE, GENERAL, PACKED, EXACT>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_grp_wg<D, TYPE, GENERAL, PACKED, EXACT>, WBLOCK, smem) !=
              hipSuccess || occ < 1)
        occ = 1;
    }
    uint64_t blocks = B->n_reads, cap = (uint64_t)ctx->n_cu * occ;
    if (blocks > cap) blocks = cap;
    if (blocks == 0) return AM_OK;
    hipLaunchKernelGGL((k_grp_wg<D, TYPE, GENERAL, PACKED, EXACT>), dim3((unsigned)blocks), dim3(WBLOCK), smem,
                       ctx->stream, *L, *B, *R, S, next);
  }
  AM_HIP(hipGetLastError());
  return AM_OK;
}

// kernel variants: the fast path (full clocks, no TxIds / bases / op ids: GENERAL false)
// over the packed view, with the n_dc == D case specialised; everything else runs GENERAL
// the group kernels' NewLastOp takes explicit op ids (a GC that kept non-consecutive ops) in
// either variant, so the op_id column alone does not need the general one
inline bool grp_batch_general(const am_op_log *L, const am_read_batch *B) {
  return L->snap_pres || (B->txid && L->op_txid) || B->base_ignore || B->per_read_clock || B->base.v0 ||
         B->base.set_off;
}

template <int D, int TYPE>
int launch_v(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S, am_retry next,
             int tier) {
  const bool general = grp_batch_general(L, B), packed = am_log_packed(L);
  if (!general && packed)
    return L->n_dc == (uint32_t)D ? launch_d<D, TYPE, false, true, true>(ctx, L, B, R, S, next, tier)
                                  : launch_d<D, TYPE, false, true, false>(ctx, L, B, R, S, next, tier);
  if (packed)  // cached bases, TxIds, per-read clocks (the vnode's read/6 path)
    return L->n_dc == (uint32_t)D ? launch_d<D, TYPE, true, true, true>(ctx, L, B, R, S, next, tier)
                                  : launch_d<D, TYPE, true, true, false>(ctx, L, B, R, S, next, tier);
  return launch_d<D, TYPE, true, false, false>(ctx, L, B, R, S, next, tier);
}

}  // namespace amk_grp
