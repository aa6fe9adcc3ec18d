// am_gc.hip -- op-cache ingestion + garbage collection on the device.
//
// The reference keeps one ETS tuple per key, {Key, {Length, ListLen}, OpCounter, Op_1..}
// (include/antidote.hrl:81-90), appends with op_insert_gc/3 (src/materializer_vnode.erl:
// 622-647: OpCounter += 1, the op stored as {NewId, Payload}) and prunes with prune_ops/2 +
// check_filter/7 (:565-604): an op survives iff materializer:belongs_to_snapshot_op(
// Threshold, CommitTime, SnapshotTime) (src/materializer.erl:102-106), i.e. it is NOT
// covered by Threshold = vectorclock:min of the retained snapshot clocks
// (snapshot_insert_gc/4, :515-563).  Survivors keep their ids and their order.
//
// On the device an op log is CSR over keys, so one batched call rebuilds it:
//   k_upd_count    one wave per key: survivor count (ballot popcounts) and payload words
//   exclusive scans (hipcub) -> new key_off / var_off bases
//   k_upd_scatter  one wave per key: survivors, then the key's new ops, copied column by
//                  column with coalesced stores (positions from ballot prefix counts)
// with the packed view (am_packop.h; the key's time base re-derived from its first output
// op) written from the same registers, then the record view
// (am_store_pack_records) of the new store.  Each column is
// read once and written once: HBM-bound stream compaction, no atomics.
//
// Deliberate differences from the ETS layout (both are ETS tuple artefacts):
//   - ListLen / RESIZE_THRESHOLD sizing does not exist: the CSR log is exactly sized.
//   - prune_ops' quirk of keeping element(FIRST_OP+Len) (a 0 "op") when every op is
//     pruned (:580-583) is reported as AM_GC_PRUNED_ALL with zero ops kept.
#include <hipcub/hipcub.hpp>

#include "am_internal.h"
#include "am_packop.h"

int am_store_pack_records(am_store *st);  // am_pack.hip

namespace {

constexpr int WAVE_SZ = 64;
constexpr uint32_t OPS_THRESHOLD = 50;  // src/materializer_vnode.erl:41

struct UpdArgs {
  am_op_log L;                 // the store's current log (device)
  am_op_log N;                 // new ops, CSR over the same keys (device); N.key_off null => none
  const uint64_t *counter;     // [n_keys] OpCounter, or null => derived from L
  const uint8_t *mask;         // [n_keys] prune this key, or null => no pruning
  const uint64_t *thr_vc;      // [n_dc][n_keys]
  const uint32_t *thr_pres;    // [n_keys]
  uint64_t *keep_bits;         // [n_ops/64 + 2] survivor bitmap of pruned keys (count -> scatter)
  uint64_t *used;              // slack layout: [n_keys] ops / [n_keys] var words the key holds
  uint64_t *vused;             //   (cnt / vcnt then hold the key's capacities); null => exact
  const uint64_t *cap_hint;    // slack layout: [n_keys] op capacity wanted per key, or null
};

// Room for appends of a slack store (the ETS tuple's ListLen slack,
// src/materializer_vnode.erl:540-560): a quarter of the key's ops and at least 4 free slots
// (one slot always stays free: var_off[key_end] ends the last op's words); variable words in
// proportion to the key's own words per op.
__device__ __forceinline__ uint64_t slack_cap(uint64_t n) {
  const uint64_t room = n / 4 > 4 ? n / 4 : 4;
  return n + room;
}
__device__ __forceinline__ uint64_t slack_vcap(uint64_t n, uint64_t nv, uint64_t cap) {
  const uint64_t per = n ? (nv + n - 1) / n : 0;
  return nv + (cap - n) * (per > 2 ? per : 2) + 4;
}

__device__ __forceinline__ uint32_t lane() { return threadIdx.x & (WAVE_SZ - 1); }

__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
  for (int o = 32; o > 0; o >>= 1) v += (uint64_t)__shfl_xor((unsigned long long)v, o, WAVE_SZ);
  return v;
}
__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t v) {
  const uint32_t l = lane();
  for (int o = 1; o < WAVE_SZ; o <<= 1) {
    const uint64_t t = (uint64_t)__shfl_up((unsigned long long)v, (unsigned)o, WAVE_SZ);
    if (l >= (uint32_t)o) v += t;
  }
  return v;
}
__device__ __forceinline__ uint64_t wave_bcast(uint64_t v, uint32_t src) {
  return (uint64_t)__shfl((unsigned long long)v, (int)src, WAVE_SZ);
}

__device__ __forceinline__ uint32_t all_mask(uint32_t n_dc) { return n_dc >= 32 ? 0xFFFFFFFFu : ((1u << n_dc) - 1u); }

// check_filter's predicate: belongs_to_snapshot_op(Thr, {Dc, CT}, SS) = not le(SS[Dc := CT], Thr)
// with vectorclock:le over keys(X) ++ keys(Thr), a missing entry reading 0.
__device__ __forceinline__ bool survives(const am_op_log &L, uint64_t p, const UpdArgs &A, uint64_t k,
                                         uint32_t tpres) {
  const uint64_t stride = L.snap_stride ? L.snap_stride : L.n_ops;
  const uint32_t all = all_mask(L.n_dc);
  const uint32_t dc = AM_META_DC(L.op_meta[p]);
  const uint32_t xpres = ((L.snap_pres ? L.snap_pres[p] : all) | (1u << dc)) & all;
  const uint64_t ct = L.commit_time[p];
  for (uint32_t d = 0; d < L.n_dc; ++d) {
    if (!((xpres >> d) & 1u)) continue;
    const uint64_t x = d == dc ? ct : L.snap_vc[(uint64_t)d * stride + p];
    const uint64_t t = ((tpres >> d) & 1u) ? A.thr_vc[(uint64_t)d * A.L.n_keys + k] : 0;
    if (x > t) return true;
  }
  return false;
}

__device__ __forceinline__ uint64_t var_len(const am_op_log &L, uint64_t p) {
  return L.var_off ? L.var_off[p + 1] - L.var_off[p] : 0;
}

__global__ void k_upd_count(UpdArgs A, uint64_t *cnt, uint64_t *vcnt) {
  const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x / WAVE_SZ);
  for (uint64_t k = (uint64_t)blockIdx.x * (blockDim.x / WAVE_SZ) + threadIdx.x / WAVE_SZ; k < A.L.n_keys; k += waves) {
    const uint64_t o0 = A.L.key_off[k], o1 = am_kend(A.L, k);
    const bool prune = A.mask && A.mask[k];
    const uint32_t tpres = prune ? A.thr_pres[k] : 0;
    uint64_t kept = 0, vk = 0;
    for (uint64_t b = o0; b < o1; b += WAVE_SZ) {
      const uint64_t p = b + lane();
      const bool in = p < o1;
      const bool keep = in && (!prune || survives(A.L, p, A, k, tpres));
      const uint64_t m = __ballot(keep);
      kept += __popcll(m);
      if (A.L.var_off) vk += wave_sum(keep ? var_len(A.L, p) : 0);
      if (prune && m) {  // chunk bits at op positions b..b+63 (two words; neighbours share them)
        const uint32_t sh = (uint32_t)(b & 63);
        if (lane() == 0) atomicOr((unsigned long long *)&A.keep_bits[b >> 6], (unsigned long long)(m << sh));
        if (lane() == 1 && sh && (m >> (64 - sh)))
          atomicOr((unsigned long long *)&A.keep_bits[(b >> 6) + 1], (unsigned long long)(m >> (64 - sh)));
      }
    }
    uint64_t nn = 0, nv = 0;
    if (A.N.key_off) {
      const uint64_t n0 = A.N.key_off[k], n1 = A.N.key_off[k + 1];
      nn = n1 - n0;
      if (A.N.var_off) nv = A.N.var_off[n1] - A.N.var_off[n0];
    }
    if (lane() == 0) {
      const uint64_t n = kept + nn, v = vk + nv;
      if (A.used) {
        uint64_t cap = slack_cap(n);
        if (A.cap_hint && A.cap_hint[k] > cap) cap = A.cap_hint[k];
        A.used[k] = n, A.vused[k] = v;
        cnt[k] = cap;
        vcnt[k] = slack_vcap(n, v, cap);
      } else {
        cnt[k] = n;
        vcnt[k] = v;
      }
    }
  }
}

// survivor bits of the pruned chunk [b, min(b + 64, o1)) from the count pass's bitmap
__device__ __forceinline__ uint64_t chunk_bits(const UpdArgs &A, uint64_t b, uint64_t o1) {
  const uint32_t sh = (uint32_t)(b & 63);
  uint64_t mb = A.keep_bits[b >> 6] >> sh;
  if (sh) mb |= A.keep_bits[(b >> 6) + 1] << (64 - sh);
  if (o1 - b < WAVE_SZ) mb &= (1ull << (o1 - b)) - 1ull;
  return mb;
}

// the packed-view time base of key k in the new log: from its first output op (the first
// survivor, else the first new op)
__device__ __forceinline__ uint64_t out_base(const UpdArgs &A, uint64_t k, uint64_t o0, uint64_t o1, bool prune) {
  const am_op_log *S = &A.L;
  uint64_t p = ~0ull;
  if (o1 > o0 && !prune) p = o0;
  for (uint64_t b = o0; prune && b < o1 && p == ~0ull; b += WAVE_SZ) {
    const uint64_t mb = chunk_bits(A, b, o1);
    if (mb) p = b + (uint64_t)__builtin_ctzll(mb);
  }
  if (p == ~0ull && A.N.key_off && A.N.key_off[k + 1] > A.N.key_off[k]) S = &A.N, p = A.N.key_off[k];
  if (p == ~0ull) return 0;
  const uint64_t ss = S->snap_stride ? S->snap_stride : S->n_ops;
  uint64_t s[AM_MAX_DC];
  for (uint32_t d = 0; d < S->n_dc; ++d) s[d] = S->snap_vc[(uint64_t)d * ss + p];
  return am_pk_base(S->commit_time[p], s, S->n_dc, 0xFFFFFFFFu, AM_META_DC(S->op_meta[p]));
}

struct OutCols {
  uint64_t *key_id_base, *counter;
  uint8_t *key_type, *key_flags, *gc_flags, *gap;
  uint8_t *op_meta;
  uint64_t *commit_time, *snap_vc;
  uint32_t *snap_pres;
  uint64_t *op_txid, *op_id, *p0, *p1, *var_off, *var_data;
  uint64_t *key_tbase;          // packed view of the new log (am_packop.h), or null
  uint32_t *pk_vc;
  uint64_t *key_end;            // slack layout: [n_keys] end of the key's ops, or null
  uint64_t stride;
};

__device__ __forceinline__ void put_op(const am_op_log &S, uint64_t p, const OutCols &O, uint64_t q, uint64_t id,
                                       uint64_t vq, uint64_t base) {
  const uint64_t ss = S.snap_stride ? S.snap_stride : S.n_ops;
  const uint32_t all = all_mask(S.n_dc);
  const uint32_t meta = S.op_meta[p];
  const uint64_t ct = S.commit_time[p];
  const uint32_t pres = S.snap_pres ? S.snap_pres[p] : all;
  O.op_meta[q] = (uint8_t)meta;
  O.commit_time[q] = ct;
  for (uint32_t d = 0; d < S.n_dc; ++d) O.snap_vc[(uint64_t)d * O.stride + q] = S.snap_vc[(uint64_t)d * ss + p];
  if (O.pk_vc)
    am_pk_write(O.pk_vc, O.stride, q, S.n_dc, base, ct, meta,
                [&](uint32_t d) { return S.snap_vc[(uint64_t)d * ss + p]; });
  if (O.snap_pres) O.snap_pres[q] = pres;
  if (O.op_txid) O.op_txid[q] = S.op_txid ? S.op_txid[p] : ~0ull;
  O.op_id[q] = id;
  O.p0[q] = S.p0[p];
  O.p1[q] = S.p1 ? S.p1[p] : 0;
  if (O.var_off) {
    O.var_off[q] = vq;
    if (S.var_off)
      for (uint64_t i = S.var_off[p], e = S.var_off[p + 1]; i < e; ++i) O.var_data[vq++] = S.var_data[i];
  }
}

// DK > 0: n_dc == DK -- every column of a chunk is loaded up front into registers (all
// loads in flight before the predicate), the survivor is written from registers.
// DK == 0: any n_dc, predicate and copy straight from memory.
template <int DK>
__global__ void k_upd_scatter(UpdArgs A, const uint64_t *cnt, const uint64_t *vcnt, OutCols O) {
  const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x / WAVE_SZ);
  const uint64_t lt = (1ull << lane()) - 1ull;
  for (uint64_t k = (uint64_t)blockIdx.x * (blockDim.x / WAVE_SZ) + threadIdx.x / WAVE_SZ; k < A.L.n_keys; k += waves) {
    const uint64_t o0 = A.L.key_off[k], o1 = am_kend(A.L, k);
    const uint64_t idb = A.L.key_id_base ? A.L.key_id_base[k] : 1;
    const uint64_t counter = A.counter ? A.counter[k]
                             : o1 > o0 ? (A.L.op_id ? A.L.op_id[o1 - 1] : idb + (o1 - o0) - 1)
                                       : idb - 1;
    const bool prune = A.mask && A.mask[k];
    uint64_t q = cnt[k], vq = vcnt[k];
    uint64_t kept = 0, first_id = 0, last_id = 0;
    constexpr int DR = DK > 0 ? DK : 1;
    const uint64_t base = O.pk_vc ? out_base(A, k, o0, o1, prune) : 0;
    if (O.key_tbase && lane() == 0) O.key_tbase[k] = base;
    const uint64_t sstride = A.L.snap_stride ? A.L.snap_stride : A.L.n_ops;
    const uint32_t all = all_mask(A.L.n_dc);
    for (uint64_t b = o0; b < o1; b += WAVE_SZ) {
      const uint64_t p = b + lane();
      const bool in = p < o1;
      // survivors of a pruned key come from the count pass's bitmap: a chunk with none is
      // skipped without touching its columns, and the predicate is not evaluated again
      const uint64_t mb = prune ? chunk_bits(A, b, o1) : 0;
      if (prune && !mb) continue;
      const bool keep = prune ? ((mb >> lane()) & 1ull) != 0 : in;
      uint64_t x[DR], ct = 0, v0 = 0, v1 = 0;
      uint32_t meta = 0, spres = all;
      if constexpr (DK > 0) {
        if (keep) {
          meta = A.L.op_meta[p];
          ct = A.L.commit_time[p];
          for (int d = 0; d < DK; ++d) x[d] = A.L.snap_vc[(uint64_t)d * sstride + p];
          v0 = A.L.p0[p];
          v1 = A.L.p1 ? A.L.p1[p] : 0;
          if (A.L.snap_pres) spres = A.L.snap_pres[p];
        }
      }
      const uint64_t m = __ballot(keep);
      if (!m) continue;
      const uint64_t vl = keep ? var_len(A.L, p) : 0;
      const uint64_t vincl = A.L.var_off ? wave_incl_scan(vl) : 0;
      const uint64_t id = in ? (A.L.op_id ? A.L.op_id[p] : idb + (p - o0)) : 0;
      if (keep) {
        const uint64_t qq = q + __popcll(m & lt);
        if constexpr (DK > 0) {
          O.op_meta[qq] = (uint8_t)meta;
          O.commit_time[qq] = ct;
          for (int d = 0; d < DK; ++d) O.snap_vc[(uint64_t)d * O.stride + qq] = x[d];
          if (O.pk_vc) am_pk_write(O.pk_vc, O.stride, qq, DK, base, ct, meta, [&](uint32_t d) { return x[d]; });
          if (O.snap_pres) O.snap_pres[qq] = spres;
          if (O.op_txid) O.op_txid[qq] = A.L.op_txid ? A.L.op_txid[p] : ~0ull;
          O.op_id[qq] = id;
          O.p0[qq] = v0;
          O.p1[qq] = v1;
          if (O.var_off) {
            uint64_t w = vq + vincl - vl;
            O.var_off[qq] = w;
            if (A.L.var_off)
              for (uint64_t i = A.L.var_off[p], e = A.L.var_off[p + 1]; i < e; ++i) O.var_data[w++] = A.L.var_data[i];
          }
        } else {
          put_op(A.L, p, O, qq, id, vq + vincl - vl, base);
        }
      }
      const uint32_t lo = __ffsll((unsigned long long)m) - 1, hi = 63 - __clzll((long long)m);
      const uint64_t id_lo = wave_bcast(id, lo), id_hi = wave_bcast(id, hi);
      if (kept == 0) first_id = id_lo;
      last_id = id_hi;
      kept += __popcll(m);
      q += __popcll(m);
      vq += wave_bcast(vincl, 63);
    }
    uint64_t nn = 0;
    uint32_t ntype = 0, nflags = 0;
    if (A.N.key_off) {
      const uint64_t n0 = A.N.key_off[k], n1 = A.N.key_off[k + 1];
      nn = n1 - n0;
      ntype = A.N.key_type ? A.N.key_type[k] : 0;
      nflags = A.N.key_flags ? A.N.key_flags[k] : 0;
      for (uint64_t b = n0; b < n1; b += WAVE_SZ) {
        const uint64_t p = b + lane();
        const bool in = p < n1;
        const uint64_t vl = in ? var_len(A.N, p) : 0;
        const uint64_t vincl = A.N.var_off ? wave_incl_scan(vl) : 0;
        // op_insert_gc: NewId = ets:update_counter(OpsCache, Key, {3, 1})
        if (in) put_op(A.N, p, O, q + lane(), counter + 1 + (p - n0), vq + vincl - vl, base);
        const uint64_t w = (n1 - b) < WAVE_SZ ? (n1 - b) : WAVE_SZ;
        q += w;
        vq += wave_bcast(vincl, 63);
      }
    }
    if (O.key_end) {  // slack: the free slots' var_off all end the key's words; their op
      const uint64_t cap_end = cnt[k + 1];  // header words are defined (zero), not reused memory
      for (uint64_t p = q + lane(); p < cap_end; p += WAVE_SZ) {
        if (O.var_off) O.var_off[p] = vq;
        O.op_meta[p] = 0;
        O.commit_time[p] = 0;
        O.p0[p] = 0;
        O.p1[p] = 0;
        // commit vectors too: the zone index's bounds over the room stay at the used ops
        for (uint32_t d = 0; d < A.L.n_dc; ++d) O.snap_vc[(uint64_t)d * O.stride + p] = 0;
        if (O.snap_pres) O.snap_pres[p] = 0;
        if (O.pk_vc)
          for (uint32_t d = 0; d < A.L.n_dc; ++d) O.pk_vc[(uint64_t)d * O.stride + p] = 0;
      }
      if (lane() == 0) O.key_end[k] = q;
    }
    if (lane() == 0) {
      const uint64_t nops_old = o1 - o0;
      const uint32_t otype = A.L.key_type[k];
      const uint32_t oflags = A.L.key_flags ? A.L.key_flags[k] : 0;
      const bool mixed = nops_old && nn && ntype != otype;
      O.key_type[k] = (uint8_t)(nops_old ? otype : (nn ? ntype : otype));
      O.key_flags[k] = (uint8_t)(oflags | nflags | (mixed ? AM_KEY_MIXED_TYPES : 0));
      O.counter[k] = counter + nn;
      O.key_id_base[k] = kept ? first_id : counter + 1;
      // ids stay dense from key_id_base iff the survivors are consecutive and end at OpCounter
      const bool gap = kept && (last_id - first_id + 1 != kept || (nn && last_id != counter));
      O.gap[k] = gap ? 1 : 0;
      uint8_t f = 0;
      if (prune && !kept) f |= AM_GC_PRUNED_ALL;  // check_filter's NewSize == 0 (:580)
      if ((counter + nn) / OPS_THRESHOLD > counter / OPS_THRESHOLD) f |= AM_GC_TRIGGER;
      if (O.gc_flags) O.gc_flags[k] = f;
    }
  }
}

unsigned grid_keys(uint64_t n_keys) {
  const uint64_t g = (n_keys + 3) / 4;  // 4 waves per 256-thread block
  return (unsigned)(g == 0 ? 1 : g < 65536 ? g : 65536);
}

}  // namespace

extern "C" int am_store_update(am_ctx *c, const am_store *st, const am_op_log *dev_new, const uint8_t *prune_mask,
                               const uint64_t *thr_vc, const uint32_t *thr_pres, uint8_t *gc_flags, am_store **out) {
  if (!c) return AM_ERR_INVALID;
  AM_LOCK(c);
  if (!c || !st || !out) return AM_ERR_INVALID;
  return am_store_update_ex(c, st->dev, st->counter, dev_new, prune_mask, thr_vc, thr_pres, gc_flags, false, nullptr,
                            out);
}

int am_store_update_ex(am_ctx *c, const am_op_log &L, const uint64_t *counter, const am_op_log *dev_new,
                       const uint8_t *prune_mask, const uint64_t *thr_vc, const uint32_t *thr_pres, uint8_t *gc_flags,
                       bool slack, const uint64_t *cap_hint, am_store **out) {
  AM_LOCK(c);
  if (prune_mask && (!thr_vc || !thr_pres)) {
    am_set_error("am_store_update: prune_mask needs thr_vc and thr_pres");
    return AM_ERR_INVALID;
  }
  if (dev_new && (!dev_new->key_off || dev_new->n_keys != L.n_keys || dev_new->n_dc != L.n_dc ||
                  (dev_new->n_ops && (!dev_new->op_meta || !dev_new->commit_time || !dev_new->snap_vc || !dev_new->p0)))) {
    am_set_error("am_store_update: the new-op log must be CSR over the store's keys with the same n_dc");
    return AM_ERR_INVALID;
  }
  AM_HIP(hipSetDevice(c->device));
  const uint64_t nk = L.n_keys;
  UpdArgs A{};
  A.L = L;
  if (dev_new) A.N = *dev_new;
  A.counter = counter;
  A.mask = prune_mask;
  A.thr_vc = thr_vc;
  A.thr_pres = thr_pres;

  // ---- pass 1: counts + exclusive scans.  Temporaries live in the context's grow-only GC
  //      scratch slot (no allocation per update once it has grown to the store's size).
  uint64_t *cnt = nullptr, *vcnt = nullptr;
  uint8_t *gap = nullptr, *gap_max = nullptr;
  void *tmp = nullptr;
  size_t tmp_b = 0, t2 = 0;
  auto cleanup = [&]() { (void)hipStreamSynchronize(c->stream); };
  if (hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_b, cnt, cnt, nk + 1, c->stream) != hipSuccess ||
      hipcub::DeviceReduce::Max(nullptr, t2, gap, gap_max, nk ? nk : 1, c->stream) != hipSuccess) {
    am_set_error("am_store_update: scan sizing failed");
    return AM_ERR_HIP;
  }
  if (t2 > tmp_b) tmp_b = t2;
  {
    const size_t o_vcnt = am_round_up((nk + 1) * 8, 256), o_gap = o_vcnt + am_round_up((nk + 1) * 8, 256);
    const size_t o_gmax = o_gap + am_round_up(nk + 1, 256), o_tmp = o_gmax + 256;
    const size_t o_keep = o_tmp + am_round_up(tmp_b + 16, 256);
    const size_t o_used = o_keep + (prune_mask ? am_round_up((L.n_ops / 64 + 2) * 8, 256) : 0);
    const size_t total = o_used + (slack ? 2 * am_round_up(nk * 8 + 8, 256) : 0);
    void *scr = nullptr;
    if (int rc = am_ctx_scratch(c, AM_SCR_GC, total, &scr)) return rc;
    char *b = (char *)scr;
    cnt = (uint64_t *)b;
    vcnt = (uint64_t *)(b + o_vcnt);
    gap = (uint8_t *)(b + o_gap);
    gap_max = (uint8_t *)(b + o_gmax);
    tmp = b + o_tmp;
    A.keep_bits = prune_mask ? (uint64_t *)(b + o_keep) : nullptr;
    A.used = slack ? (uint64_t *)(b + o_used) : nullptr;
    A.cap_hint = slack ? cap_hint : nullptr;
    A.vused = slack ? (uint64_t *)(b + o_used + am_round_up(nk * 8 + 8, 256)) : nullptr;
  }
  uint64_t tot[2] = {0, 0};
  bool ok = hipMemsetAsync(cnt + nk, 0, 8, c->stream) == hipSuccess &&
            hipMemsetAsync(vcnt + nk, 0, 8, c->stream) == hipSuccess &&
            hipMemsetAsync(gap, 0, nk + 1, c->stream) == hipSuccess &&
            (!A.keep_bits || hipMemsetAsync(A.keep_bits, 0, (L.n_ops / 64 + 2) * 8, c->stream) == hipSuccess);
  if (ok && nk) {
    hipLaunchKernelGGL(k_upd_count, dim3(grid_keys(nk)), dim3(256), 0, c->stream, A, cnt, vcnt);
    ok = hipGetLastError() == hipSuccess;
  }
  ok = ok && hipcub::DeviceScan::ExclusiveSum(tmp, tmp_b, cnt, cnt, nk + 1, c->stream) == hipSuccess &&
       hipcub::DeviceScan::ExclusiveSum(tmp, tmp_b, vcnt, vcnt, nk + 1, c->stream) == hipSuccess &&
       hipMemcpyAsync(&tot[0], cnt + nk, 8, hipMemcpyDeviceToHost, c->stream) == hipSuccess &&
       hipMemcpyAsync(&tot[1], vcnt + nk, 8, hipMemcpyDeviceToHost, c->stream) == hipSuccess &&
       hipStreamSynchronize(c->stream) == hipSuccess;
  if (!ok) {
    cleanup();
    am_set_error("am_store_update: count pass failed");
    return AM_ERR_HIP;
  }
  const uint64_t n_out = tot[0], v_out = tot[1];

  // ---- the new store's columns (padded like am_store_create)
  am_store *ns = new am_store();
  ns->ctx = c;
  am_op_log &d = ns->dev;
  const uint64_t na = am_round_up(n_out, AM_OP_PAD) + AM_OP_PAD;
  const bool has_pres = L.snap_pres || (dev_new && dev_new->snap_pres);
  const bool has_txid = L.op_txid || (dev_new && dev_new->op_txid);
  const bool has_var = L.var_off || (dev_new && dev_new->var_off);
  d.n_dc = L.n_dc;
  d.n_keys = nk;
  d.n_ops = n_out;
  d.n_var = has_var ? v_out : 0;
  d.snap_stride = na;
  int rc = AM_OK;
  // every element below `used` is written by k_upd_scatter; only the pad tail is zeroed
  auto alloc = [&](size_t bytes, size_t used) -> void * {
    void *p = nullptr;
    if (rc) return nullptr;
    rc = am_dev_alloc(c, bytes, &p);
    if (rc) return nullptr;
    ns->allocs.push_back(p);
    if (bytes > used && hipMemsetAsync((char *)p + used, 0, bytes - used, c->stream) != hipSuccess) rc = AM_ERR_HIP;
    return p;
  };
  OutCols O{};
  O.stride = na;
  O.key_id_base = (uint64_t *)alloc(nk * 8 + 8, nk * 8);
  O.counter = (uint64_t *)alloc(nk * 8 + 8, nk * 8);
  O.key_type = (uint8_t *)alloc(nk + 8, nk);
  O.key_flags = (uint8_t *)alloc(nk + 8, nk);
  O.gc_flags = gc_flags;
  O.gap = gap;
  O.op_meta = (uint8_t *)alloc(na, n_out);
  O.commit_time = (uint64_t *)alloc(na * 8, n_out * 8);
  O.snap_vc = (uint64_t *)alloc((size_t)L.n_dc * na * 8, (size_t)L.n_dc * na * 8);  // DC tails zeroed below
  O.snap_pres = has_pres ? (uint32_t *)alloc(na * 4, n_out * 4) : nullptr;
  O.op_txid = has_txid ? (uint64_t *)alloc(na * 8, n_out * 8) : nullptr;
  O.op_id = (uint64_t *)alloc(na * 8, n_out * 8);
  O.p0 = (uint64_t *)alloc(na * 8, n_out * 8);
  O.p1 = (uint64_t *)alloc(na * 8, n_out * 8);
  O.var_off = has_var ? (uint64_t *)alloc((n_out + 1) * 8, (n_out + 1) * 8) : nullptr;
  O.var_data = has_var ? (uint64_t *)alloc(v_out * 8 + 32, v_out * 8) : nullptr;
  if (!has_pres) {  // the packed view needs full clocks (am_pack.hip)
    O.key_tbase = (uint64_t *)alloc(nk * 8 + 8, nk * 8);
    O.pk_vc = (uint32_t *)alloc((size_t)L.n_dc * na * 4, (size_t)L.n_dc * na * 4);  // DC tails zeroed below
  }
  uint64_t *key_off = (uint64_t *)alloc((nk + 1) * 8, (nk + 1) * 8);
  O.key_end = slack ? (uint64_t *)alloc(nk * 8 + 8, nk * 8) : nullptr;
  for (uint32_t dd = 0; !rc && dd < L.n_dc && na > n_out; ++dd)
    if (hipMemsetAsync(O.snap_vc + (uint64_t)dd * na + n_out, 0, (na - n_out) * 8, c->stream) != hipSuccess ||
        (O.pk_vc && hipMemsetAsync(O.pk_vc + (uint64_t)dd * na + n_out, 0, (na - n_out) * 4, c->stream) != hipSuccess))
      rc = AM_ERR_HIP;
  if (rc) {
    cleanup();
    am_store_destroy(ns);
    return rc;
  }
  uint8_t any_gap = 0;
  ok = hipMemcpyAsync(key_off, cnt, (nk + 1) * 8, hipMemcpyDeviceToDevice, c->stream) == hipSuccess;
  if (ok && has_var) ok = hipMemcpyAsync(O.var_off + n_out, vcnt + nk, 8, hipMemcpyDeviceToDevice, c->stream) == hipSuccess;
  if (ok && nk) {
    const dim3 g(grid_keys(nk)), t(256);
    switch (L.n_dc) {
      case 1: hipLaunchKernelGGL(k_upd_scatter<1>, g, t, 0, c->stream, A, cnt, vcnt, O); break;
      case 2: hipLaunchKernelGGL(k_upd_scatter<2>, g, t, 0, c->stream, A, cnt, vcnt, O); break;
      case 3: hipLaunchKernelGGL(k_upd_scatter<3>, g, t, 0, c->stream, A, cnt, vcnt, O); break;
      case 4: hipLaunchKernelGGL(k_upd_scatter<4>, g, t, 0, c->stream, A, cnt, vcnt, O); break;
      default: hipLaunchKernelGGL(k_upd_scatter<0>, g, t, 0, c->stream, A, cnt, vcnt, O); break;
    }
    ok = hipGetLastError() == hipSuccess;
  }
  ok = ok && hipcub::DeviceReduce::Max(tmp, tmp_b, gap, gap_max, nk ? nk : 1, c->stream) == hipSuccess &&
       hipMemcpyAsync(&any_gap, gap_max, 1, hipMemcpyDeviceToHost, c->stream) == hipSuccess &&
       hipStreamSynchronize(c->stream) == hipSuccess;
  cleanup();
  if (!ok) {
    am_store_destroy(ns);
    am_set_error("am_store_update: scatter pass failed");
    return AM_ERR_HIP;
  }
  d.key_off = key_off;
  d.key_end = O.key_end;
  d.key_id_base = O.key_id_base;
  d.key_type = O.key_type;
  d.key_flags = O.key_flags;
  d.op_meta = O.op_meta;
  d.commit_time = O.commit_time;
  d.snap_vc = O.snap_vc;
  d.snap_pres = O.snap_pres;
  d.op_txid = O.op_txid;
  d.op_id = any_gap ? O.op_id : nullptr;  // dense ids keep the kernels on their fast paths
  d.p0 = O.p0;
  d.p1 = O.p1;
  d.var_off = O.var_off;
  d.var_data = O.var_data;
  d.key_tbase = O.key_tbase;
  d.pk_vc = O.pk_vc;
  ns->counter = O.counter;
  rc = am_store_pack_records(ns);  // the packed view was written by k_upd_scatter
  if (rc) {
    am_store_destroy(ns);
    return rc;
  }
  *out = ns;
  return AM_OK;
}
