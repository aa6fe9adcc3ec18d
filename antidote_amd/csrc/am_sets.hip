// am_sets.hip -- materialize/4 for the order-sensitive CRDTs (add-wins set,
// MV register) and the bounded counter.  One 256-thread workgroup per read.
//
// antidote_crdt_set_aw / antidote_crdt_register_mv apply their effects
// sequentially (oldest -> newest), but the final state has a closed form that
// needs no sequential fold.  Call every token an effect inserts a BIRTH at the
// op's position p (AW: {Elem, Tok} for each Add token; MV: {Value, Tok}) and
// every token it drops a KILL at p (AW: {Elem, Tok} for each Remove token; MV:
// each Overridden token).  Within one effect the AW update is
// ToAdd ++ (Current -- ToRemove) and the MV update removes Overridden before
// inserting, so a kill only affects births at earlier positions:
//     a birth at p survives  <=>  no kill of the same token (and AW: elem) at q > p
// Base-snapshot pairs are births at p = -1.  The workgroup therefore
//   1. streams the key's log in 1024-op tiles (4 ops per lane, 16-byte loads),
//      evaluates inclusion per op (am_wave.h eval_op), and appends the included
//      effects' births / kills to LDS lists (LDS atomics for the slots);
//   2. bitonic-sorts the kills by (token, elem, pos) in LDS;
//   3. keeps each birth whose upper-bound lookup finds no later kill;
//   4. bitonic-sorts the survivors into the reference's order and writes the CSR:
//      AW (elem, newest birth first, the effect's token order; base tokens last, in
//      base order) -- the orddict's token lists are ToAdd ++ (Current -- ToRemove);
//      MV (value, token) with duplicates dropped (insert_sorted).
// This tier serves the keys the token-group tier (am_group.hip) does not: base-snapshot
// reads, logs outside the group view's limits, and logs that re-add a live token (where
// it emits every surviving birth, as the list semantics do unless a later remove takes
// only one of the copies).
// The bounded counter (orddict:update_counter on P[{From,To}] and D[Id]) is a
// keyed sum: exact 128-bit LDS accumulators (64-bit atomics + carry).
// Capacity: KCAP kills / BCAP births per read live in LDS (78 KB per group);
// a read that exceeds them returns AM_ERR_CAPACITY (global-scratch path: next).
#include "am_block.h"

using namespace amk;

namespace {

constexpr int BLOCK = 256;
constexpr int NW = BLOCK / WAVE;
constexpr int OPL = 4;
constexpr uint64_t TILE = (uint64_t)BLOCK * OPL;
constexpr uint32_t KCAP = 2048;
constexpr uint32_t BCAP = 1024;
constexpr uint64_t BIG_OPS = AM_SETS_BIG_OPS;  // logs longer than this skip the LDS tier
static_assert(BIG_OPS == 4 * TILE, "the LDS tier takes logs of up to four tiles");

struct Smem {
  uint64_t *ka, *kb;  // kills: token, elem (MV: 0)
  int32_t *kp;        // kill position
  uint64_t *ba, *bb;  // births: AW (elem, tok), MV (value, tok)
  int32_t *bp;        // birth: (position + 1) << 16 | index in the effect's ToAdd / base list
  uint64_t *oa, *ob;  // survivors
  uint32_t *ctr;      // [0] kills [1] births [2] survivors [3] overflow [4..7] wave sums
  uint64_t *red;      // block reduction scratch [NW][8]
  // bounded counter slots (aliases the kill arrays)
  uint64_t *slo;
  int64_t *shi;
  uint32_t *spres;
};

// births / kills appended to the LDS lists; overflow sets ctr[3] (-> big-read tier)
// packed birth position: op position (-1 = base snapshot) and the index within the
// effect's token list (base: within the base list), for the AW output order
__device__ __forceinline__ int32_t bpack(int32_t pos, uint32_t sub) {
  return (int32_t)(((uint32_t)(pos + 1) << 16) | (sub < 0xFFFFu ? sub : 0xFFFFu));
}
__device__ __forceinline__ int32_t bpos(int32_t bp) { return (int32_t)((uint32_t)bp >> 16) - 1; }
// AW output order within one elem: newest birth first, then the effect's token order
__device__ __forceinline__ uint64_t bord(int32_t bp) {
  return ((uint64_t)(uint32_t)(0x7FFFFFFF - bpos(bp)) << 32) | ((uint32_t)bp & 0xFFFFu);
}

struct LdsSink {
  Smem *s;
  __device__ void births(uint64_t e, const uint64_t *tok, uint32_t n, int32_t pos) {
    const uint32_t bi = atomicAdd(&s->ctr[1], n);
    if (bi + n > BCAP) {
      s->ctr[3] = 1;
      return;
    }
    for (uint32_t i = 0; i < n; ++i) s->ba[bi + i] = e, s->bb[bi + i] = tok[i], s->bp[bi + i] = bpack(pos, i);
  }
  __device__ void birth(uint64_t a, uint64_t b, int32_t pos) {
    const uint32_t bi = atomicAdd(&s->ctr[1], 1u);
    if (bi >= BCAP) {
      s->ctr[3] = 1;
      return;
    }
    s->ba[bi] = a, s->bb[bi] = b, s->bp[bi] = bpack(pos, 0);
  }
  __device__ void kills(const uint64_t *tok, uint32_t n, uint64_t e, int32_t pos) {
    const uint32_t ki = atomicAdd(&s->ctr[0], n);
    if (ki + n > KCAP) {
      s->ctr[3] = 1;
      return;
    }
    for (uint32_t i = 0; i < n; ++i) s->ka[ki + i] = tok[i], s->kb[ki + i] = e, s->kp[ki + i] = pos;
  }
};

__device__ Smem carve(unsigned char *p) {
  Smem s;
  s.ka = (uint64_t *)p;
  s.kb = s.ka + KCAP;
  s.kp = (int32_t *)(s.kb + KCAP);
  s.ba = (uint64_t *)(s.kp + KCAP);
  s.bb = s.ba + BCAP;
  s.bp = (int32_t *)(s.bb + BCAP);
  s.oa = (uint64_t *)(s.bp + BCAP);
  s.ob = s.oa + BCAP;
  s.ctr = (uint32_t *)(s.ob + BCAP);
  s.red = (uint64_t *)(s.ctr + 16);
  s.slo = s.ka;
  s.shi = (int64_t *)s.kb;
  s.spres = (uint32_t *)s.kp;
  return s;
}
constexpr size_t SMEM_BYTES = (size_t)KCAP * 20 + (size_t)BCAP * 20 + (size_t)BCAP * 16 + 16 * 4 + NW * 8 * 8;

template <int DMAX, int TYPE, bool PACKED>
__global__ void __launch_bounds__(BLOCK) k_sets(am_op_log L, am_read_batch B, am_read_result R, am_sel S,
                                                am_retry retry) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  Smem s = carve(smem_raw);
  const uint32_t tid = threadIdx.x;
  const uint64_t n = B.n_reads;
  const uint32_t nd = L.n_dc;
  const uint32_t np = nd * nd;
  const uint64_t stride = L.snap_stride ? L.snap_stride : L.n_ops;

  const uint32_t sel0 = S.idx ? uniform_u32(S.range[0]) : 0u;
  const uint64_t nsel = S.idx ? (uint64_t)(uniform_u32(S.range[1]) - sel0) : n;
  for (uint64_t i = blockIdx.x; i < nsel; i += gridDim.x) {
    const uint64_t r = S.idx ? (uint64_t)uniform_u32(S.idx[sel0 + i]) : i;
    const uint64_t key = uniform_u64(B.key[r]);
    const uint32_t rtype = uniform_u32(B.type[r]);
    int32_t status = AM_OK;
    uint64_t off0 = 0, off1 = 0;
    if (key >= L.n_keys) {
      status = AM_ERR_INVALID;
    } else {
      off0 = uniform_u64(L.key_off[key]);
      off1 = uniform_u64(am_kend(L, key));
      const uint32_t ktype = uniform_u32(L.key_type[key]);
      const uint32_t kfl = L.key_flags ? uniform_u32(L.key_flags[key]) : 0u;
      if (off1 > off0 && (ktype != rtype || (kfl & AM_KEY_MIXED_TYPES))) status = AM_ERR_CORRUPTED_OPS_CACHE;
      else if (rtype != (uint32_t)TYPE) status = AM_ERR_INVALID;
    }
    if (status != AM_OK) {
      if (tid == 0) R.status[r] = status;
      continue;
    }
    // A log far beyond the LDS tier goes straight to the big-read path (am_big.hip).
    // So does a hot MV key with the chunked token-group view (its grouped mode there streams u32
    // records instead of var_data).
    const bool big_grp = TYPE == AM_MVREG && L.key_ngrp && am_ngrp_big(uniform_u32(L.key_ngrp[key])) &&
                         !(B.base.set_off && B.base.set_len[r]);
    if (retry.list && (off1 - off0 > BIG_OPS || big_grp)) {
      if (tid == 0) retry.list[atomicAdd(retry.count, 1u)] = (uint32_t)r;
      continue;
    }

    // ---- per-read uniform inputs ----
    ReadU<DMAX> u;
    u.allmask = nd >= 32 ? 0xFFFFFFFFu : ((1u << nd) - 1u);
    const uint64_t rstride = B.per_read_clock ? n : 1, ridx = B.per_read_clock ? r : 0;
    u.spres = uniform_u32(B.read_pres[ridx]) & u.allmask;
    u.base_ignore = !B.base_ignore || B.base_ignore[r];
    u.cpres = u.base_ignore ? 0u : (uniform_u32(B.base_pres[r]) & u.allmask);
#pragma unroll
    for (int d = 0; d < DMAX; ++d) {
      u.S[d] = (d < (int)nd && ((u.spres >> d) & 1u)) ? uniform_u64(B.read_vc[(uint64_t)d * rstride + ridx]) : 0;
      u.C0[d] = (d < (int)nd && ((u.cpres >> d) & 1u)) ? uniform_u64(B.base_vc[(uint64_t)d * n + r]) : 0;
    }
    u.has_txid = B.txid && (!B.txid_valid || B.txid_valid[r]) && L.op_txid;
    u.txid = u.has_txid ? uniform_u64(B.txid[r]) : 0;

    if (tid < 16) s.ctr[tid] = 0;
    if (TYPE == AM_BCOUNTER) {
      for (uint32_t i = tid; i < np + nd; i += BLOCK) {
        uint32_t bpres = 0;
        const int64_t bv = bc_base(B, r, np, nd, i, bpres);
        s.slo[i] = (uint64_t)bv;
        s.shi[i] = bv < 0 ? -1 : 0;
        s.spres[i] = bpres;
      }
    }
    __syncthreads();
    if (TYPE != AM_BCOUNTER && B.base.set_off) {  // base snapshot pairs: births at -1
      const uint64_t bo = B.base.set_off[r];
      const uint32_t bl = B.base.set_len[r];
      if (bl > BCAP) {
        if (tid == 0) s.ctr[3] = 1;
      } else {
        for (uint32_t i = tid; i < bl; i += BLOCK) {
          s.ba[i] = B.base.set_a[bo + i];
          s.bb[i] = B.base.set_b[bo + i];
          s.bp[i] = bpack(-1, i);
        }
        if (tid == 0) s.ctr[1] = bl;
      }
    }
    __syncthreads();

    Acc<DMAX> a;
    a.reset();
    AccP<DMAX> ap;
    ap.reset();
    PkRead<DMAX> pk;
    if (PACKED) pk_setup(u, nd, uniform_u64(L.key_tbase[key]), pk);
    LdsSink sink{&s};
    // ---- stream the log, 1024 ops per tile ----
    for (uint64_t t0 = off0 & ~(uint64_t)(OPL - 1); t0 < off1; t0 += TILE) {
      const uint64_t g = t0 + (uint64_t)tid * OPL;
      if (g < off1) {
        const uint32_t meta4 = *(const uint32_t *)(L.op_meta + g);
        uint32_t ib = 0;
        if constexpr (PACKED) {
          ib = incl4<DMAX, true>(L, nd, stride, u, pk, g, off0, off1, ap, a);
        } else {
          const u64x2 c01 = *(const u64x2 *)(L.commit_time + g), c23 = *(const u64x2 *)(L.commit_time + g + 2);
          const uint64_t ct[OPL] = {c01.x, c01.y, c23.x, c23.y};
          uint64_t sv[OPL][DMAX];
#pragma unroll
          for (int d = 0; d < DMAX; ++d) {
            if (d < (int)nd) {
              const uint64_t *col = L.snap_vc + (uint64_t)d * stride + g;
              const u64x2 s01 = *(const u64x2 *)col, s23 = *(const u64x2 *)(col + 2);
              sv[0][d] = s01.x, sv[1][d] = s01.y, sv[2][d] = s23.x, sv[3][d] = s23.y;
            } else {
              sv[0][d] = sv[1][d] = sv[2][d] = sv[3][d] = 0;
            }
          }
          uint32_t sp[OPL] = {u.allmask, u.allmask, u.allmask, u.allmask};
          if (L.snap_pres) {
            const u32x4 q = *(const u32x4 *)(L.snap_pres + g);
            sp[0] = q.x, sp[1] = q.y, sp[2] = q.z, sp[3] = q.w;
          }
#pragma unroll
          for (int k = 0; k < OPL; ++k) {
            const uint64_t p = g + k;
            if (p < off0 || p >= off1) continue;
            const bool txm = u.has_txid && L.op_txid[p] == u.txid;
            if (eval_op<DMAX, true>(u, (meta4 >> (8 * k)) & 0xFFu, ct[k], sv[k], sp[k], txm, p, a)) ib |= 1u << k;
          }
        }
#pragma unroll
        for (int k = 0; k < OPL; ++k) {
          if (!((ib >> k) & 1u)) continue;
          const uint64_t p = g + k;
          const uint32_t meta = (meta4 >> (8 * k)) & 0xFFu;
          if (meta & AM_META_BAD) continue;  // reported through FLAG_BAD
          const int32_t pos = (int32_t)(p - off0);
          if (TYPE == AM_BCOUNTER) {
            uint32_t slot;
            int64_t v;
            if (!bc_slot(L, p, meta, nd, slot, v)) {
              a.flags |= FLAG_BAD;
              continue;
            }
            acc128_atomic(&s.slo[slot], &s.shi[slot], v < 0 ? -1 : 0, (uint64_t)v);
            atomicOr(&s.spres[slot], 1u);
          } else if (!set_effects<TYPE>(L, p, meta, pos, sink)) {
            a.flags |= FLAG_BAD;
          }
        }
      }
    }
    if (PACKED) pk_fold(ap, pk.K, u.allmask, a);
    __syncthreads();

    // ---- scalar outputs (block reductions) ----
    const uint32_t count = (uint32_t)block_red_u64(s.red, wave_sum_u32(a.count), 0);
    const uint32_t flags = (uint32_t)block_red_u64(s.red, wave_or_u32(a.flags), 1);
    const uint32_t pres = (uint32_t)block_red_u64(s.red, wave_or_u32(a.pres), 1);
    const uint64_t min_excl = block_red_u64(s.red, wave_min_u64(a.min_excl), 3);
    uint64_t mx[DMAX];
#pragma unroll
    for (int d = 0; d < DMAX; ++d) mx[d] = d < (int)nd ? block_red_u64(s.red, wave_max_u64(a.mx[d]), 2) : 0;
    status = (flags & FLAG_BAD) ? AM_ERR_UNEXPECTED_OPERATION : AM_OK;
    if (status == AM_OK && s.ctr[3]) {
      if (retry.list) {  // the births/kills did not fit in LDS: hand the read to am_big.hip
        if (tid == 0) retry.list[atomicAdd(retry.count, 1u)] = (uint32_t)r;
        __syncthreads();
        continue;
      }
      status = AM_ERR_CAPACITY;
    }

    if (status == AM_OK && TYPE == AM_BCOUNTER) {
      uint32_t *ovf = &s.ctr[8];  // no static __shared__: keeps the dynamic LDS base 16-byte aligned
      if (tid == 0) *ovf = 0;
      __syncthreads();
      for (uint32_t i = tid; i < np + nd; i += BLOCK) {
        const uint64_t lo = s.slo[i];
        const int64_t hi = s.shi[i];
        if (hi != ((int64_t)lo < 0 ? -1 : 0)) atomicOr(ovf, 1u);
      }
      __syncthreads();
      if (*ovf) {
        status = AM_ERR_OVERFLOW;
      } else {
        if (tid < WAVE) {  // one wave compacts the present slots into the read's CSR range
          const uint32_t ne = bc_emit<WAVE>(R, r, np + nd, tid, 0, [&](uint32_t k, int64_t &v) {
            v = (int64_t)s.slo[k];
            return s.spres[k] != 0;
          });
          if (tid == 0) *ovf = ne;
        }
        __syncthreads();
        const uint32_t ne = *ovf;
        if (ne > R.value.set_off[r + 1] - R.value.set_off[r]) status = AM_ERR_CAPACITY;
        else if (tid == 0) R.value.set_len[r] = ne;
        __syncthreads();
      }
    }
    if (status == AM_OK && TYPE != AM_BCOUNTER) {
      const uint32_t nk = s.ctr[0], nb = s.ctr[1];
      block_sort(s.ka, s.kb, s.kp, nk, KCAP);  // by (token, elem, pos)
      if (tid == 0) s.ctr[2] = 0;
      __syncthreads();
      for (uint32_t i = tid; i < nb; i += BLOCK) {
        // kill key of this birth: AW (tok, elem), MV (tok, 0)
        const uint64_t qa = s.bb[i], qb = TYPE == AM_AWSET ? s.ba[i] : 0;
        // upper bound of (qa, qb, +inf)
        uint32_t lo = 0, hi = nk;
        while (lo < hi) {
          const uint32_t mid = (lo + hi) >> 1;
          const bool le = s.ka[mid] < qa || (s.ka[mid] == qa && s.kb[mid] <= qb);
          if (le) lo = mid + 1;
          else hi = mid;
        }
        bool alive = true;
        if (lo > 0 && s.ka[lo - 1] == qa && s.kb[lo - 1] == qb) alive = s.kp[lo - 1] <= bpos(s.bp[i]);
        if (!alive) s.bp[i] = -1;  // dead (packed positions are >= 0)
      }
      __syncthreads();
      // survivors: AW keyed (elem, output order) with the token in the (free) kill arrays,
      // MV keyed (value, token)
      for (uint32_t i = tid; i < nb; i += BLOCK) {
        if (s.bp[i] < 0) continue;
        const uint32_t o = atomicAdd(&s.ctr[2], 1u);
        s.oa[o] = s.ba[i];
        if (TYPE == AM_AWSET) {
          s.ob[o] = bord(s.bp[i]);
          s.ka[o] = s.bb[i];
          s.kp[o] = (int32_t)o;
        } else {
          s.ob[o] = s.bb[i];
        }
      }
      __syncthreads();
      const uint32_t no = s.ctr[2];
      const uint64_t ooff = R.value.set_off[r], ocap = R.value.set_off[r + 1] - ooff;
      uint32_t base;
      if (TYPE == AM_AWSET) {
        block_sort(s.oa, s.ob, s.kp, no, BCAP);
        for (uint32_t j = tid; j < no && j < ocap; j += BLOCK) {
          R.value.set_a[ooff + j] = s.oa[j];
          R.value.set_b[ooff + j] = s.ka[s.kp[j]];
        }
        base = no;
      } else {
        block_sort(s.oa, s.ob, nullptr, no, BCAP);
        base = block_write_unique(s.oa, s.ob, no, R.value.set_a + ooff, R.value.set_b + ooff, ocap, &s.ctr[4]);
      }
      if (base > ocap) status = AM_ERR_CAPACITY;
      else if (tid == 0) R.value.set_len[r] = base;
    }

    if (tid == 0) {
      R.status[r] = status;
      R.flags[r] = (uint8_t)(flags & 0xFFu);
      if (status == AM_OK) {
        const uint64_t idb = L.key_id_base ? L.key_id_base[key] : 1;
        const uint64_t nops = off1 - off0;
        int64_t nlo;
        if (min_excl != NONE)
          nlo = (L.op_id ? (int64_t)L.op_id[min_excl] : (int64_t)(idb + (min_excl - off0))) - 1;
        else
          nlo = nops == 0 ? 0 : (L.op_id ? (int64_t)L.op_id[off1 - 1] : (int64_t)(idb + nops - 1));
        R.new_last_op[r] = nlo;
        const bool ign = u.base_ignore && count == 0;
        const uint32_t opres = ign ? 0u : (pres | u.cpres);
        R.last_ct_ignore[r] = ign ? 1 : 0;
        R.last_ct_pres[r] = opres;
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
    __syncthreads();
  }
}

// A mixed batch whose result lacks this type's value columns: its reads of the type
// (if any; the count lives on the device) fail with AM_ERR_INVALID.
__global__ void k_sets_nocols(am_read_result R, am_sel S) {
  const uint32_t b0 = S.range[0], b1 = S.range[1];
  for (uint32_t i = b0 + blockIdx.x * blockDim.x + threadIdx.x; i < b1; i += gridDim.x * blockDim.x)
    R.status[S.idx[i]] = AM_ERR_INVALID;
}

template <int TYPE>
int launch_sets(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S,
                am_retry retry) {
  const bool cols = TYPE == AM_BCOUNTER
                        ? (R->value.set_off && R->value.set_len && R->value.set_a && R->value.set_b)
                        : (R->value.set_off && R->value.set_len && R->value.set_a && R->value.set_b);
  if (!cols && S.idx) {
    hipLaunchKernelGGL(k_sets_nocols, dim3(64), dim3(256), 0, ctx->stream, *R, S);
    AM_HIP(hipGetLastError());
    return AM_OK;
  }
  if (!cols) {
    am_set_error(TYPE == AM_BCOUNTER ? "bcounter results need value.set_off/set_len/set_a/set_b"
                                     : "set results need value.set_off/set_len/set_a/set_b");
    return AM_ERR_INVALID;
  }
  if (TYPE == AM_BCOUNTER && (size_t)L->n_dc * L->n_dc + L->n_dc > KCAP) {
    am_set_error("bcounter: n_dc too large for the LDS slots");
    return AM_ERR_UNSUPPORTED;
  }
  uint64_t blocks = B->n_reads;
  const uint64_t cap = (uint64_t)ctx->n_cu * 2;  // 2 groups per CU (78 KB LDS each)
  if (blocks > cap) blocks = cap;
  if (blocks == 0) return AM_OK;
  const uint32_t nd = L->n_dc;
  const bool packed = am_log_packed(L);
#define AM_SP(D, P)                                                                                    \
  {                                                                                                    \
    static bool attr = false;                                                                          \
    if (!attr) {                                                                                       \
      AM_HIP(hipFuncSetAttribute((const void *)k_sets<D, TYPE, P>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                 (int)SMEM_BYTES));                                                    \
      attr = true;                                                                                     \
    }                                                                                                  \
    hipLaunchKernelGGL((k_sets<D, TYPE, P>), dim3((unsigned)blocks), dim3(BLOCK), SMEM_BYTES, ctx->stream, \
                       *L, *B, *R, S, retry);                                                          \
  }
#define AM_S(D)          \
  if (packed) AM_SP(D, true) \
  else AM_SP(D, false)   \
  break;
  switch (nd <= 1 ? 1 : nd <= 2 ? 2 : nd <= 3 ? 3 : nd <= 4 ? 4 : nd <= 8 ? 8 : nd <= 16 ? 16 : 32) {
    case 1: AM_S(1)
    case 2: AM_S(2)
    case 3: AM_S(3)
    case 4: AM_S(4)
    case 8: AM_S(8)
    case 16: AM_S(16)
    default: AM_S(32)
  }
#undef AM_S
#undef AM_SP
  AM_HIP(hipGetLastError());
  return AM_OK;
}

}  // namespace

int am_launch_sets(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S,
                   uint32_t type, am_retry retry) {
  switch (type) {
    case AM_AWSET: return launch_sets<AM_AWSET>(ctx, L, B, R, S, retry);
    case AM_MVREG: return launch_sets<AM_MVREG>(ctx, L, B, R, S, retry);
    case AM_BCOUNTER: return launch_sets<AM_BCOUNTER>(ctx, L, B, R, S, retry);
    default: return AM_ERR_UNSUPPORTED;
  }
}
