// am_block.h -- workgroup-level building blocks of the set-CRDT kernels (256 threads):
// bitonic sort of (a, b, pos) triples and scalar reductions.  The sort works on LDS or,
// for the big-read tier, on global scratch (__syncthreads orders both for the group).
#pragma once
#include "am_wave.h"

namespace amk {

constexpr int SBLOCK = 256;
constexpr int32_t POS_MAX = 0x7FFFFFFF;

__device__ __forceinline__ bool less3(uint64_t a0, uint64_t b0, int32_t p0, uint64_t a1, uint64_t b1, int32_t p1) {
  return a0 != a1 ? a0 < a1 : (b0 != b1 ? b0 < b1 : p0 < p1);
}

// ascending bitonic sort of (a, b, p) by (a, b, p); n <= cap, padded to a power of two
// with +inf (the arrays must hold next_pow2(n) entries)
__device__ void block_sort(uint64_t *a, uint64_t *b, int32_t *p, uint32_t n, uint32_t cap) {
  uint32_t N = 1;
  while (N < n) N <<= 1;
  if (N > cap) N = cap;
  for (uint32_t i = n + threadIdx.x; i < N; i += SBLOCK) {
    a[i] = ~0ull;
    b[i] = ~0ull;
    if (p) p[i] = POS_MAX;
  }
  __syncthreads();
  for (uint32_t k = 2; k <= N; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t i = threadIdx.x; i < N; i += SBLOCK) {
        const uint32_t x = i ^ j;
        if (x > i) {
          const bool up = (i & k) == 0;
          const int32_t pi = p ? p[i] : 0, px = p ? p[x] : 0;
          const bool gt = less3(a[x], b[x], px, a[i], b[i], pi);
          if (gt == up) {
            uint64_t t = a[i]; a[i] = a[x]; a[x] = t;
            t = b[i]; b[i] = b[x]; b[x] = t;
            if (p) { const int32_t q = p[i]; p[i] = p[x]; p[x] = q; }
          }
        }
      }
      __syncthreads();
    }
  }
}

// block-wide reduction of per-wave values (DPP wave reductions first); red = 4 u64 of LDS
__device__ __forceinline__ uint64_t block_red_u64(uint64_t *red, uint64_t wave_val, int op /*0 sum,1 or,2 max,3 min*/) {
  const uint32_t w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = wave_val;
  __syncthreads();
  uint64_t r = red[0];
  for (int i = 1; i < SBLOCK / WAVE; ++i) {
    const uint64_t x = red[i];
    r = op == 0 ? r + x : op == 1 ? (r | x) : op == 2 ? (r > x ? r : x) : (r < x ? r : x);
  }
  __syncthreads();
  return r;
}

// Write the sorted pairs (oa, ob)[0, no) to the read's CSR slot, dropping duplicates
// (the state is a set rendered in Erlang term order).  ctr4 = 4 u32 of LDS.  Returns
// the distinct count (uniform); entries beyond the caller's capacity are not written.
__device__ uint32_t block_write_unique(const uint64_t *oa, const uint64_t *ob, uint32_t no, uint64_t *out_a,
                                       uint64_t *out_b, uint64_t ocap, uint32_t *ctr4) {
  const uint32_t tid = threadIdx.x;
  uint32_t base = 0;
  for (uint32_t c = 0; c < no; c += SBLOCK) {
    const uint32_t i = c + tid;
    const bool keep = i < no && (i == 0 || oa[i] != oa[i - 1] || ob[i] != ob[i - 1]);
    const uint64_t m = __ballot(keep);
    const uint32_t w = tid >> 6, l = tid & 63;
    const uint32_t before = __popcll(m & ((1ull << l) - 1));
    if (l == 0) ctr4[w] = __popcll(m);
    __syncthreads();
    uint32_t woff = 0;
    for (uint32_t k = 0; k < w; ++k) woff += ctr4[k];
    const uint32_t total = ctr4[0] + ctr4[1] + ctr4[2] + ctr4[3];
    if (keep) {
      const uint32_t o = base + woff + before;
      if (o < ocap) {
        out_a[o] = oa[i];
        out_b[o] = ob[i];
      }
    }
    base += total;
    __syncthreads();
  }
  return base;
}

// The effects of one included op as births / kills (see am_sets.hip):
//   MV  {Value, Token, Overridden}: kills (tok, 0) for each overridden token, then a
//       birth (value, tok); {reset, Overridden} only kills
//   AW  [{Elem, AddTokens, RemoveTokens}]: births (elem, tok) per add token, kills
//       (tok, elem) per remove token
// Sink: births(a, const uint64_t *b, n, pos) (n pairs (a, b[i])), birth(a, b, pos),
// kills(const uint64_t *tok, n, elem, pos).  Returns false for a malformed effect
// (Type:update/2 would raise: {error, {unexpected_operation, ...}}).
template <int TYPE, class Sink>
__device__ __forceinline__ bool set_effects(const am_op_log &L, uint64_t p, uint32_t meta, int32_t pos, Sink &sk) {
  const uint64_t vo = L.var_off ? L.var_off[p] : 0, ve = L.var_off ? L.var_off[p + 1] : 0;
  if (TYPE == AM_MVREG) {
    if (ve > vo) sk.kills(L.var_data + vo, (uint32_t)(ve - vo), 0ull, pos);
    if (AM_META_KIND(meta) != AM_MV_RESET) sk.birth(L.p0[p], L.p1[p], pos);
    return true;
  }
  uint64_t q = vo;  // AW-set entries [elem, n_add, n_rm, add..., rm...]
  while (q < ve) {
    if (q + 3 > ve) return false;
    const uint64_t e = L.var_data[q], na = L.var_data[q + 1], nr = L.var_data[q + 2];
    if (na > ve - q || nr > ve - q || q + 3 + na + nr > ve) return false;
    if (na) sk.births(e, L.var_data + q + 3, (uint32_t)na, pos);
    if (nr) sk.kills(L.var_data + q + 3 + na, (uint32_t)nr, e, pos);
    q += 3 + na + nr;
  }
  return true;
}

// bounded counter effect -> slot (P {From,To} at From*D+To, D Id at D*D+Id); false when
// malformed.  orddict:update_counter is a keyed sum: accumulate v into the slot.
__device__ __forceinline__ bool bc_slot(const am_op_log &L, uint64_t p, uint32_t meta, uint32_t nd, uint32_t &slot,
                                        int64_t &v) {
  const uint32_t kind = AM_META_KIND(meta);
  const uint32_t from = (uint32_t)(L.p1[p] & 0xFF), to = (uint32_t)((L.p1[p] >> 8) & 0xFF);
  if (kind > AM_BC_TRANSFER || from >= nd || to >= nd) return false;
  slot = kind == AM_BC_DECREMENT ? nd * nd + from : from * nd + (kind == AM_BC_INCREMENT ? from : to);
  v = (int64_t)L.p0[p];
  return true;
}
// exact 128-bit accumulation with 64-bit atomics (LDS or global): lo += v, hi += sign + carry
__device__ __forceinline__ void acc128_atomic(uint64_t *lo, int64_t *hi, int64_t vhi, uint64_t vlo) {
  const uint64_t old = atomicAdd((unsigned long long *)lo, (unsigned long long)vlo);
  const int64_t carry = (old + vlo < old) ? 1 : 0;
  if (vhi + carry) atomicAdd((unsigned long long *)hi, (unsigned long long)(vhi + carry));
}

// kill key of a birth (a, b): AW (tok, elem) = (b, a); MV (tok, 0) = (b, 0)
template <int TYPE>
__device__ __forceinline__ void birth_kill_key(uint64_t a, uint64_t b, uint64_t &ka, uint64_t &kb) {
  ka = b;
  kb = TYPE == AM_AWSET ? a : 0ull;
}

}  // namespace amk
