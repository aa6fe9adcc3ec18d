// am_apply.hip -- op-cache ingestion + GC in place, for the keys a batch touches:
// materializer_vnode:op_insert_gc/3 appends (src/materializer_vnode.erl:622-647) and
// snapshot_insert_gc/4's prune_ops/2 of one key (:515-604) at O(the touched keys' ops), not a
// whole-store rebuild.
//
// A vnode store keeps room for appends per key (key_end / rec_key_end in am_op_log: the ETS
// tuple's ListLen slack, :540-560).  am_store_apply:
//   1. k_view: the touched keys as a log of m keys over the store's OWN op columns (key ranges
//      and per-key columns gathered; no op is copied);
//   2. the ordinary rebuild on that view (am_store_update_ex: prune, append with ids
//      OpCounter+1.., packed view, token-group view) -> a small dense store of the touched keys;
//   3. k_fit: every touched key still fits its room (ops + one free slot, variable words,
//      records); one u32 readback.  If a key does not fit nothing is written and the caller
//      rebuilds the whole store, regrowing every key's room (the reference doubles ListLen);
//   4. k_writeback, one wave per key: every op column, the packed view under the key's new time
//      base, the variable words (offsets rebased), the records and group pairs, the key's
//      header (end, OpCounter, id base, type, flags, group count).
// Readers take a key's end from key_end (am_kend), so the free slots behind it are never read.
#include "am_wave.h"

namespace {
using amk::wave_max_u64;
using amk::wave_sync;

constexpr int WAVE_SZ = 64;

struct ViewCols {
  uint64_t *off, *end, *idb, *ctr;
  uint8_t *type, *flags;
};

// per touched key: its range and header in the store -> the view's columns
// (a key outside the store reads as key 0: the caller's key check fails the call before any
// write)
__global__ void k_view(am_op_log L, const uint64_t *counter, const uint64_t *keys, uint64_t m, ViewCols V) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t k = keys[i] < L.n_keys ? keys[i] : 0;
    V.off[i] = L.key_off[k];
    V.end[i] = am_kend(L, k);
    V.idb[i] = L.key_id_base ? L.key_id_base[k] : 1;
    V.type[i] = L.key_type[k];
    V.flags[i] = L.key_flags ? L.key_flags[k] : 0;
    if (counter) V.ctr[i] = counter[k];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) V.off[m] = 0;
}

// thr_vc [n_dc][n_keys] / thr_pres [n_keys] of the store's keys -> [n_dc][m] / [m]
__global__ void k_thr_gather(const uint64_t *keys, uint64_t m, uint32_t n_dc, uint64_t n_keys, const uint8_t *mask,
                             const uint64_t *thr_vc, const uint32_t *thr_pres, uint8_t *omask, uint64_t *ovc,
                             uint32_t *opres) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t k = keys[i] < n_keys ? keys[i] : 0;
    omask[i] = mask[k];
    opres[i] = thr_pres[k];
    for (uint32_t d = 0; d < n_dc; ++d) ovc[(uint64_t)d * m + i] = thr_vc[(uint64_t)d * n_keys + k];
  }
}

__device__ __forceinline__ bool set_type(uint32_t t) { return t == AM_AWSET || t == AM_MVREG; }

// does key i of the rebuilt view S fit key keys[i]'s room in L?
__global__ void k_fit(am_op_log L, am_op_log S, const uint64_t *keys, uint64_t m, uint32_t *nofit) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t k = keys[i] < L.n_keys ? keys[i] : 0;
    const uint64_t c0 = L.key_off[k], c1 = L.key_off[k + 1];
    const uint64_t s0 = S.key_off[i], s1 = S.key_off[i + 1];
    bool ok = s1 - s0 + 1 <= c1 - c0;
    if (ok && L.var_off) ok = (S.var_off ? S.var_off[s1] - S.var_off[s0] : 0) <= L.var_off[c1] - L.var_off[c0];
    if (ok && L.rec_key_off && S.rec_key_off && set_type(S.key_type[i]))
      ok = am_rkend(S, i) - S.rec_key_off[i] <= L.rec_key_off[k + 1] - L.rec_key_off[k];
    if (!ok) atomicOr(nofit, 1u);
  }
}

// the first record of S's key range [r0, r1) (op order) whose op is >= relative op `rel`
__device__ __forceinline__ uint64_t rec_lower_s(const am_op_log &S, uint64_t r0, uint64_t r1, uint64_t rel) {
  while (r0 < r1) {
    const uint64_t mid = (r0 + r1) >> 1;
    if (AM_REC_OP(S.rec_g[mid]) < rel) r0 = mid + 1;
    else r1 = mid;
  }
  return r0;
}

// the zone index of the blocks inside store key k's op range [d0, cap_end) (room included),
// from the rebuilt key i of S written at d0: maxima over the used slots, the exact mark (every
// slot a used op, none escaped / invalid; zlevel >= AM_INDEX_EXACT), and the group summary
// rewritten into the block's slot when the key's new group count fits it (else retired: row
// n_dc + 1 = ~0).  One wave; no other key shares these blocks.
__device__ void zone_rewrite(const am_op_log &L, const am_op_log &S, uint64_t i, uint64_t d0, uint64_t n,
                             uint64_t cap_end, uint64_t r0, int zlevel, uint32_t lane, uint32_t *bw) {
  const uint64_t ls = L.snap_stride ? L.snap_stride : L.n_ops, ss = S.snap_stride ? S.snap_stride : S.n_ops;
  const uint64_t nz = (ls + AM_ZONE_OPS - 1) / AM_ZONE_OPS;
  const uint32_t nd = L.n_dc;
  uint64_t *Z = const_cast<uint64_t *>(L.zone_vc);
  const uint64_t s0 = S.key_off[i];
  const uint32_t t = S.key_type[i];
  const uint32_t ng = (S.rec_key_off && S.key_ngrp) ? S.key_ngrp[i] : AM_NGRP_NONE, G = am_ngrp_count(ng);
  const bool grouped = L.zone_gsum && (t == AM_AWSET || t == AM_MVREG) && !am_ngrp_big(ng) && G >= 1 &&
                       G <= AM_GRP_MAX_REC;
  const uint32_t gw = (G + 31) / 32;
  for (uint64_t z = (d0 + AM_ZONE_OPS - 1) / AM_ZONE_OPS; (z + 1) * AM_ZONE_OPS <= cap_end; ++z) {
    const uint64_t z0 = z * AM_ZONE_OPS;
    bool ok = zlevel >= AM_INDEX_EXACT && z0 + AM_ZONE_OPS <= d0 + n && S.pk_vc && L.pk_vc;
    uint64_t mx[AM_MAX_DC];
    for (uint32_t d = 0; d < nd; ++d) mx[d] = 0;
    for (uint64_t q = z0 + lane; q < z0 + AM_ZONE_OPS; q += WAVE_SZ) {
      if (q >= d0 + n) continue;  // free room: never read
      const uint64_t p = s0 + (q - d0);
      const uint32_t meta = S.op_meta[p], dc = AM_META_DC(meta);
      const uint32_t sp = S.snap_pres ? S.snap_pres[p] : 0xFFFFFFFFu;
      for (uint32_t d = 0; d < nd; ++d) {
        const uint64_t x = d == dc ? S.commit_time[p] : (((sp >> d) & 1u) ? S.snap_vc[(uint64_t)d * ss + p] : 0);
        mx[d] = x > mx[d] ? x : mx[d];
      }
      if (S.pk_vc && (S.pk_vc[p] == AM_PK_ESC || (meta & AM_META_BAD))) ok = false;
    }
    for (uint32_t d = 0; d < nd; ++d) {
      const uint64_t m = wave_max_u64(mx[d]);
      if (lane == 0) Z[(uint64_t)d * nz + z] = m;
    }
    const bool exact = __ballot(!ok) == 0;
    if (lane == 0) Z[(uint64_t)nd * nz + z] = exact ? 1u : 0u;
    const uint64_t slot = Z[(uint64_t)(nd + 4) * nz + z];
    const uint64_t cap = slot >> 48, o = slot & ((1ull << 48) - 1);
    if (!(exact && grouped && slot && 2 * (uint64_t)gw <= cap)) {
      if (lane == 0) Z[(uint64_t)(nd + 1) * nz + z] = ~0ull;
      continue;
    }
    const uint64_t sr0 = S.rec_key_off[i], sr1 = am_rkend(S, i);
    const uint64_t rb = rec_lower_s(S, sr0, sr1, z0 - d0), re = rec_lower_s(S, sr0, sr1, z0 + AM_ZONE_OPS - d0);
    for (uint32_t w = lane; w < 2 * gw; w += WAVE_SZ) bw[w] = 0;
    wave_sync();
    for (uint64_t q = rb + lane; q < re; q += WAVE_SZ) {
      const uint32_t x = S.rec_g[q], g = AM_REC_GRP(x);
      if (x != 0xFFFFFFFFu) atomicOr(bw + ((x & AM_REC_KILL) ? gw : 0u) + (g >> 5), 1u << (g & 31));
    }
    wave_sync();
    uint32_t *gs = const_cast<uint32_t *>(L.zone_gsum);
    for (uint32_t w = lane; w < 2 * gw; w += WAVE_SZ) gs[o + w] = bw[w];
    if (lane == 0) {
      Z[(uint64_t)(nd + 1) * nz + z] = o;
      Z[(uint64_t)(nd + 2) * nz + z] = r0 + (re - sr0);
      Z[(uint64_t)(nd + 3) * nz + z] = r0 + (rb - sr0);
    }
    wave_sync();
  }
}

// one wave per touched key: S's key i -> the store's key keys[i]
__global__ void __launch_bounds__(256) k_writeback(am_op_log L, am_op_log S, const uint64_t *s_counter,
                                                   uint64_t *counter, const uint64_t *keys, uint64_t m, int zlevel) {
  __shared__ uint32_t zbits[4][2 * (AM_GRP_MAX_REC / 32)];  // per wave: a block's summary being rebuilt
  const uint32_t lane = threadIdx.x & (WAVE_SZ - 1);
  const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x / WAVE_SZ);
  const uint64_t ls = L.snap_stride ? L.snap_stride : L.n_ops, ss = S.snap_stride ? S.snap_stride : S.n_ops;
  uint8_t *op_meta = const_cast<uint8_t *>(L.op_meta);
  uint64_t *commit_time = const_cast<uint64_t *>(L.commit_time), *snap_vc = const_cast<uint64_t *>(L.snap_vc);
  uint64_t *p0 = const_cast<uint64_t *>(L.p0), *p1 = const_cast<uint64_t *>(L.p1);
  for (uint64_t i = (uint64_t)blockIdx.x * (blockDim.x / WAVE_SZ) + threadIdx.x / WAVE_SZ; i < m; i += waves) {
    const uint64_t k = keys[i];
    const uint64_t d0 = L.key_off[k], cap_end = L.key_off[k + 1];
    const uint64_t s0 = S.key_off[i], n = S.key_off[i + 1] - s0;
    const uint64_t idb = S.key_id_base ? S.key_id_base[i] : 1;
    const uint64_t vb = L.var_off ? L.var_off[d0] : 0, sv0 = S.var_off ? S.var_off[s0] : 0;
    const uint64_t nv = S.var_off ? S.var_off[s0 + n] - sv0 : 0;
    for (uint64_t j = lane; j < n; j += WAVE_SZ) {
      const uint64_t p = s0 + j, q = d0 + j;
      op_meta[q] = S.op_meta[p];
      commit_time[q] = S.commit_time[p];
      for (uint32_t d = 0; d < L.n_dc; ++d) snap_vc[(uint64_t)d * ls + q] = S.snap_vc[(uint64_t)d * ss + p];
      if (L.snap_pres) const_cast<uint32_t *>(L.snap_pres)[q] = S.snap_pres ? S.snap_pres[p] : 0xFFFFFFFFu;
      if (L.op_txid) const_cast<uint64_t *>(L.op_txid)[q] = S.op_txid ? S.op_txid[p] : ~0ull;
      if (L.op_id) const_cast<uint64_t *>(L.op_id)[q] = S.op_id ? S.op_id[p] : idb + j;
      p0[q] = S.p0[p];
      p1[q] = S.p1 ? S.p1[p] : 0;
      if (L.pk_vc && S.pk_vc) {
        for (uint32_t d = 0; d < L.n_dc; ++d)
          const_cast<uint32_t *>(L.pk_vc)[(uint64_t)d * ls + q] = S.pk_vc[(uint64_t)d * ss + p];
        // an escaped op written here reads the columns (its row index is S's, not the store's)
        if (L.n_dc >= 2 && S.pk_vc[p] == AM_PK_ESC) const_cast<uint32_t *>(L.pk_vc)[ls + q] = 0;
      }
      if (L.lag_ct) {  // the lag view under the key's new lag bases (S's; escaped without them)
        const bool lv = S.lag_ct && S.lag && S.key_lag;
        const_cast<uint32_t *>(L.lag_ct)[q] = lv ? S.lag_ct[p] : AM_PK_ESC;
        for (uint32_t d = 0; d < L.n_dc; ++d)
          const_cast<uint16_t *>(L.lag)[(uint64_t)d * ls + q] = lv ? S.lag[(uint64_t)d * ss + p] : 0;
      }
      if (L.var_off) const_cast<uint64_t *>(L.var_off)[q] = vb + (S.var_off ? S.var_off[p] - sv0 : 0);
      if (L.gmask) const_cast<uint64_t *>(L.gmask)[q] = S.gmask ? S.gmask[p] : 0;
      const uint64_t zq = q / AM_ZONE_OPS;
      if (L.zone_vc && !(zq * AM_ZONE_OPS >= d0 && (zq + 1) * AM_ZONE_OPS <= cap_end)) {
        // a block shared with another key: its bound stays an upper bound of the ops written
        const uint64_t nz = (ls + AM_ZONE_OPS - 1) / AM_ZONE_OPS;
        const uint32_t dc = AM_META_DC(S.op_meta[p]), sp = S.snap_pres ? S.snap_pres[p] : 0xFFFFFFFFu;
        for (uint32_t d = 0; d < L.n_dc; ++d) {
          const uint64_t x = d == dc ? S.commit_time[p] : (((sp >> d) & 1u) ? S.snap_vc[(uint64_t)d * ss + p] : 0);
          atomicMax((unsigned long long *)const_cast<uint64_t *>(L.zone_vc) + (uint64_t)d * nz + zq,
                    (unsigned long long)x);
        }
      }
    }
    for (uint64_t q = d0 + n + lane; L.gmask && q < cap_end; q += WAVE_SZ) const_cast<uint64_t *>(L.gmask)[q] = 0;
    if (L.key_lag)
      for (uint32_t d = lane; d < L.n_dc; d += WAVE_SZ)
        const_cast<int32_t *>(L.key_lag)[k * L.n_dc + d] = (S.key_lag && S.lag_ct) ? S.key_lag[i * S.n_dc + d] : 0;
    if (L.zone_vc)  // the blocks inside the key: maxima, marks and summaries recomputed
      zone_rewrite(L, S, i, d0, n, cap_end, L.rec_key_off ? L.rec_key_off[k] : 0, zlevel, lane,
                   zbits[threadIdx.x / WAVE_SZ]);
    if (L.var_off) {
      uint64_t *vo = const_cast<uint64_t *>(L.var_off);
      for (uint64_t q = d0 + n + lane; q < cap_end; q += WAVE_SZ) vo[q] = vb + nv;  // the free slots
      uint64_t *vd = const_cast<uint64_t *>(L.var_data);
      for (uint64_t w = lane; w < nv; w += WAVE_SZ) vd[vb + w] = S.var_data[sv0 + w];
    }
    const uint32_t t = S.key_type[i];
    uint32_t ng = set_type(t) ? 0u : AM_NGRP_NONE;
    if (L.rec_key_off) {
      const uint64_t r0 = L.rec_key_off[k];
      uint64_t nr = 0;
      if (S.rec_key_off && S.key_ngrp) {
        const uint64_t sr0 = S.rec_key_off[i];
        nr = am_rkend(S, i) - sr0;
        ng = S.key_ngrp[i];
        uint32_t *rg = const_cast<uint32_t *>(L.rec_g);
        for (uint64_t r = lane; r < nr; r += WAVE_SZ) rg[r0 + r] = S.rec_g[sr0 + r];
        if (L.prec && S.prec) {  // the birth-ordered pairs travel with their records
          uint64_t *pr = const_cast<uint64_t *>(L.prec);
          for (uint64_t r = lane; r < nr; r += WAVE_SZ) {
            pr[2 * (r0 + r)] = S.prec[2 * (sr0 + r)];
            pr[2 * (r0 + r) + 1] = S.prec[2 * (sr0 + r) + 1];
          }
        }
        uint64_t *gp = const_cast<uint64_t *>(L.grp);
        const uint32_t ngc = am_ngrp_count(ng);
        for (uint32_t g = lane; g < ngc; g += WAVE_SZ) {
          gp[2 * (r0 + g)] = S.grp[2 * (sr0 + g)];
          gp[2 * (r0 + g) + 1] = S.grp[2 * (sr0 + g) + 1];
        }
      }
      if (lane == 0) {
        const_cast<uint64_t *>(L.rec_key_end)[k] = r0 + nr;
        const_cast<uint32_t *>(L.key_ngrp)[k] = ng;
      }
    }
    if (lane == 0) {
      const_cast<uint64_t *>(L.key_end)[k] = d0 + n;
      if (L.key_tbase) const_cast<uint64_t *>(L.key_tbase)[k] = S.key_tbase ? S.key_tbase[i] : 0;
      const_cast<uint8_t *>(L.key_type)[k] = (uint8_t)t;
      if (L.key_flags) const_cast<uint8_t *>(L.key_flags)[k] = S.key_flags ? S.key_flags[i] : 0;
      if (L.key_id_base) const_cast<uint64_t *>(L.key_id_base)[k] = idb;
      if (counter) counter[k] = s_counter[i];
    }
  }
}

// dense op ids (key_id_base + position) / "no TxId" words for every used slot of a store
// that had no such column: the first gap in a key's ids (a GC that kept non-consecutive ops) or
// the first TxId turns the column on, once, for the whole store
__global__ void k_fill_ids(am_op_log L, uint64_t *op_id, uint64_t *op_txid) {
  const uint32_t lane = threadIdx.x & (WAVE_SZ - 1);
  const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x / WAVE_SZ);
  for (uint64_t k = (uint64_t)blockIdx.x * (blockDim.x / WAVE_SZ) + threadIdx.x / WAVE_SZ; k < L.n_keys; k += waves) {
    const uint64_t o0 = L.key_off[k], o1 = am_kend(L, k), idb = L.key_id_base ? L.key_id_base[k] : 1;
    for (uint64_t p = o0 + lane; p < o1; p += WAVE_SZ) {
      if (op_id) op_id[p] = idb + (p - o0);
      if (op_txid) op_txid[p] = ~0ull;
    }
  }
}

// the caller's key list: every key in range and none twice (a claim bit per store key); bad |=
// AM_BADKEY_RANGE for a key >= n_keys, AM_BADKEY_DUP for a repeated key
constexpr uint32_t AM_BADKEY_RANGE = 2u, AM_BADKEY_DUP = 4u;
__global__ void k_check_keys(const uint64_t *keys, uint64_t m, uint64_t n_keys, uint32_t *claim, uint32_t *bad) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t k = keys[i];
    if (k >= n_keys) {
      atomicOr(bad, AM_BADKEY_RANGE);
      continue;
    }
    const uint32_t bit = 1u << (k & 31);
    if (atomicOr(&claim[k >> 5], bit) & bit) atomicOr(bad, AM_BADKEY_DUP);
  }
}

unsigned grid_threads(uint64_t n) { return (unsigned)((n + 255) / 256 < 65536 ? ((n + 255) / 256 ? (n + 255) / 256 : 1) : 65536); }
unsigned grid_waves(uint64_t n) { return (unsigned)((n + 3) / 4 < 65536 ? ((n + 3) / 4 ? (n + 3) / 4 : 1) : 65536); }

}  // namespace

// the caller's key list checked the synchronous way (stores am_store_apply_ex does not update
// in place)
int check_keys_sync(am_ctx *c, const am_store *st, uint64_t m, const uint64_t *keys) {
  const uint64_t words = (st->dev.n_keys + 31) / 32;
  void *scr = nullptr;
  if (int rc = am_dev_alloc(c, words * 4 + 256, &scr)) return rc;
  uint32_t *bad = (uint32_t *)scr, *claim = bad + 64;
  uint64_t w = 0;
  int rc = hipMemsetAsync(scr, 0, words * 4 + 256, c->stream) == hipSuccess ? AM_OK : AM_ERR_HIP;
  if (!rc) {
    hipLaunchKernelGGL(k_check_keys, dim3(grid_threads(m)), dim3(256), 0, c->stream, keys, m, st->dev.n_keys, claim,
                       bad);
    rc = hipGetLastError() == hipSuccess ? AM_OK : AM_ERR_HIP;
  }
  if (!rc) rc = am_ctx_fetch(c, bad, 1, &w);
  (void)hipStreamSynchronize(c->stream);
  am_dev_release(c, scr);
  if (rc) {
    am_set_error("am_store_apply: key check failed");
    return rc;
  }
  if (w & (AM_BADKEY_RANGE | AM_BADKEY_DUP)) {
    am_set_error("am_store_apply: %s", (w & AM_BADKEY_RANGE) ? "a touched key is outside the store's key space"
                                                             : "a touched key appears twice in the list");
    return AM_ERR_INVALID;
  }
  return AM_OK;
}

int am_store_apply_ex(am_ctx *c, am_store *st, uint64_t m, const uint64_t *d_keys, const am_op_log *dev_new,
                   const uint8_t *d_mask_full, const uint64_t *d_thr_vc_full, const uint32_t *d_thr_pres_full,
                   uint8_t *d_gc_flags, uint64_t *h_new_len, int *applied, bool check_keys) {
  AM_LOCK(c);
  *applied = 0;
  am_op_log &L = st->dev;
  // in place needs the slack layout with its per-key header columns and OpCounter
  const bool inplace = L.key_end && L.key_id_base && st->counter && !(L.rec_key_off && !L.rec_key_end) && m &&
                       !(dev_new && (dev_new->n_keys != m || (dev_new->snap_pres && !L.snap_pres) ||
                                     (dev_new->var_off && !L.var_off)));
  if (!inplace) return (check_keys && m) ? check_keys_sync(c, st, m, d_keys) : AM_OK;
  AM_HIP(hipSetDevice(c->device));
  const uint64_t nd = L.n_dc;
  // scratch: the view's columns, the gathered prune arguments, the fit / key-check word, the
  // key claim bitmap
  const size_t o_end = am_round_up((m + 1) * 8, 256), o_idb = o_end + am_round_up(m * 8, 256);
  const size_t o_ctr = o_idb + am_round_up(m * 8, 256), o_type = o_ctr + am_round_up(m * 8, 256);
  const size_t o_flags = o_type + am_round_up(m, 256), o_mask = o_flags + am_round_up(m, 256);
  const size_t o_tvc = o_mask + am_round_up(m, 256), o_tpres = o_tvc + am_round_up(nd * m * 8, 256);
  const size_t o_fit = o_tpres + am_round_up(m * 4, 256), o_claim = o_fit + 256;
  const size_t claim_b = check_keys ? am_round_up((L.n_keys + 31) / 32 * 4, 256) : 0, total = o_claim + claim_b + 256;
  void *scr = nullptr;
  if (int rc = am_dev_alloc(c, total, &scr)) return rc;
  char *b = (char *)scr;
  ViewCols V{(uint64_t *)b, (uint64_t *)(b + o_end), (uint64_t *)(b + o_idb), (uint64_t *)(b + o_ctr),
             (uint8_t *)(b + o_type), (uint8_t *)(b + o_flags)};
  uint8_t *mask = d_mask_full ? (uint8_t *)(b + o_mask) : nullptr;
  uint64_t *tvc = (uint64_t *)(b + o_tvc);
  uint32_t *tpres = (uint32_t *)(b + o_tpres), *nofit = (uint32_t *)(b + o_fit);
  auto done = [&](int rc) {
    (void)hipStreamSynchronize(c->stream);
    am_dev_release(c, scr);
    return rc;
  };
  if (check_keys) {  // into the fit word: one readback covers both
    if (hipMemsetAsync(b + o_fit, 0, 256 + claim_b, c->stream) != hipSuccess) {
      am_set_error("am_store_apply: key check failed");
      return done(AM_ERR_HIP);
    }
    hipLaunchKernelGGL(k_check_keys, dim3(grid_threads(m)), dim3(256), 0, c->stream, d_keys, m, L.n_keys,
                       (uint32_t *)(b + o_claim), nofit);
  }
  hipLaunchKernelGGL(k_view, dim3(grid_threads(m)), dim3(256), 0, c->stream, L, (const uint64_t *)st->counter, d_keys,
                     m, V);
  if (mask)
    hipLaunchKernelGGL(k_thr_gather, dim3(grid_threads(m)), dim3(256), 0, c->stream, d_keys, m, L.n_dc, L.n_keys,
                       d_mask_full, d_thr_vc_full, d_thr_pres_full, mask, tvc, tpres);
  if (hipGetLastError() != hipSuccess || (!check_keys && hipMemsetAsync(nofit, 0, 4, c->stream) != hipSuccess)) {
    am_set_error("am_store_apply: view failed");
    return done(AM_ERR_HIP);
  }
  am_op_log view = L;  // the touched keys over the store's own op columns
  view.n_keys = m;
  view.key_off = V.off, view.key_end = V.end, view.key_id_base = V.idb, view.key_type = V.type, view.key_flags = V.flags;
  view.key_tbase = nullptr, view.rec_key_off = nullptr, view.rec_key_end = nullptr, view.key_ngrp = nullptr;
  view.gmask = nullptr, view.zone_vc = nullptr, view.zone_gsum = nullptr, view.prec = nullptr;
  view.esc_rows = nullptr, view.lag_ct = nullptr, view.lag = nullptr, view.key_lag = nullptr;
  am_store *sub = nullptr;
  int rc = am_store_update_ex(c, view, V.ctr, dev_new, mask, mask ? tvc : nullptr, mask ? tpres : nullptr, d_gc_flags,
                              false, nullptr, &sub);
  if (rc) {
    if (check_keys) {  // a bad key list is the caller's error, whatever it did to the rebuild
      uint64_t w = 0;
      if (am_ctx_fetch(c, nofit, 1, &w) == AM_OK && (w & (AM_BADKEY_RANGE | AM_BADKEY_DUP))) rc = AM_ERR_INVALID;
      if (rc == AM_ERR_INVALID) am_set_error("am_store_apply: a touched key is outside the store or repeated");
    }
    return done(rc);
  }
  const am_op_log &S = sub->dev;
  bool cols = !(S.snap_pres && !L.snap_pres) && !(S.var_off && !L.var_off) && !(L.pk_vc && !S.pk_vc) &&
              !(S.rec_key_off && !L.rec_key_off) && !(S.gmask && !L.gmask);
  uint64_t fit = 0;
  if (cols || check_keys) {
    if (cols) hipLaunchKernelGGL(k_fit, dim3(grid_threads(m)), dim3(256), 0, c->stream, L, S, d_keys, m, nofit);
    if (hipGetLastError() != hipSuccess) rc = AM_ERR_HIP;
    uint64_t w = 0;
    if (!rc) rc = am_ctx_fetch(c, nofit, 1, &w);
    if (!rc && (w & (AM_BADKEY_RANGE | AM_BADKEY_DUP))) {
      am_set_error("am_store_apply: %s", (w & AM_BADKEY_RANGE) ? "a touched key is outside the store's key space"
                                                               : "a touched key appears twice in the list");
      rc = AM_ERR_INVALID;
    }
    fit = cols && (w & 0xFFFFFFFFull) == 0;
  }
  // a column the store lacks (its first gap in op ids, its first TxId) is turned on only once the
  // key check and the fit have passed: a failing call writes nothing into the store
  if (!rc && fit && ((S.op_id && !L.op_id) || (S.op_txid && !L.op_txid))) {  // turn the column on (O(store), once)
    const size_t na = L.snap_stride ? L.snap_stride : L.n_ops;
    void *ids = nullptr, *tx = nullptr;
    if (S.op_id && !L.op_id && !rc) rc = am_dev_alloc(c, na * 8 + 8, &ids);
    if (S.op_txid && !L.op_txid && !rc) rc = am_dev_alloc(c, na * 8 + 8, &tx);
    if (!rc && L.n_keys)
      hipLaunchKernelGGL(k_fill_ids, dim3(grid_waves(L.n_keys)), dim3(256), 0, c->stream, L, (uint64_t *)ids,
                         (uint64_t *)tx);
    if (!rc && hipGetLastError() != hipSuccess) rc = AM_ERR_HIP;
    if (rc) {
      am_dev_release(c, ids);
      am_dev_release(c, tx);
      am_store_destroy(sub);
      return done(rc);
    }
    if (ids) st->allocs.push_back(ids), L.op_id = (const uint64_t *)ids;
    if (tx) st->allocs.push_back(tx), L.op_txid = (const uint64_t *)tx;
  }
  if (!rc && fit) {
    hipLaunchKernelGGL(k_writeback, dim3(grid_waves(m)), dim3(256), 0, c->stream, L, S,
                       (const uint64_t *)sub->counter, st->counter, d_keys, m, st->zone_level);
    if (hipGetLastError() != hipSuccess) rc = AM_ERR_HIP;
    if (!rc && h_new_len) {
      std::vector<uint64_t> so(m + 1);
      if (hipMemcpyAsync(so.data(), S.key_off, (m + 1) * 8, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
          hipStreamSynchronize(c->stream) != hipSuccess)
        rc = AM_ERR_HIP;
      for (uint64_t i = 0; !rc && i < m; ++i) h_new_len[i] = so[i + 1] - so[i];
    }
    if (!rc) *applied = 1;
  }
  if (rc == AM_ERR_HIP) am_set_error("am_store_apply: device pass failed");
  rc = done(rc);
  am_store_destroy(sub);
  return rc;
}

namespace {
__global__ void k_key_lens(am_op_log L, const uint64_t *keys, uint64_t m, const uint8_t *flags_full, uint64_t *len,
                           uint8_t *flags) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t k = keys[i];
    len[i] = am_kend(L, k) - L.key_off[k];
    if (flags_full) flags[i] = flags_full[k];
  }
}
}  // namespace

// the op counts of keys[0..m) (device list) and, if flags_full [n_keys] is given, their entries
// -> host arrays
int am_store_key_lens(am_ctx *c, const am_store *st, uint64_t m, const uint64_t *d_keys, const uint8_t *flags_full,
                      uint64_t *h_len, uint8_t *h_flags) {
  AM_LOCK(c);
  if (m == 0) return AM_OK;
  void *scr = nullptr;
  if (int rc = am_dev_alloc(c, m * 9 + 64, &scr)) return rc;
  uint64_t *len = (uint64_t *)scr;
  uint8_t *fl = (uint8_t *)scr + m * 8;
  hipLaunchKernelGGL(k_key_lens, dim3(grid_threads(m)), dim3(256), 0, c->stream, st->dev, d_keys, m, flags_full, len,
                     fl);
  bool ok = hipGetLastError() == hipSuccess &&
            hipMemcpyAsync(h_len, len, m * 8, hipMemcpyDeviceToHost, c->stream) == hipSuccess &&
            (!flags_full || hipMemcpyAsync(h_flags, fl, m, hipMemcpyDeviceToHost, c->stream) == hipSuccess) &&
            hipStreamSynchronize(c->stream) == hipSuccess;
  am_dev_release(c, scr);
  if (!ok) {
    am_set_error("am_store_key_lens failed");
    return AM_ERR_HIP;
  }
  return AM_OK;
}

namespace {
// the store's keys [0, n_old) and new empty keys [n_old, n_new) as one view's key columns
__global__ void k_grow_view(am_op_log L, const uint64_t *counter, uint64_t n_new, uint64_t *off, uint64_t *end,
                            uint64_t *idb, uint64_t *ctr, uint8_t *type, uint8_t *flags) {
  const uint64_t n_old = L.n_keys, tail = L.key_off[n_old];
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k <= n_new; k += (uint64_t)gridDim.x * blockDim.x) {
    const bool old = k < n_old;
    off[k] = old ? L.key_off[k] : tail;
    if (k == n_new) continue;
    end[k] = old ? am_kend(L, k) : tail;
    idb[k] = old ? (L.key_id_base ? L.key_id_base[k] : 1) : 1;
    ctr[k] = old ? (counter ? counter[k] : 0) : 0;
    type[k] = old ? L.key_type[k] : (uint8_t)AM_PN;
    flags[k] = old ? (L.key_flags ? L.key_flags[k] : 0) : 0;
  }
}
}  // namespace

// a copy of st over n_new >= n_keys keys (the new keys empty: ets:insert of their tuple comes
// with their first op, src/materializer_vnode.erl:624-629), with room for appends
int am_store_grow_keys(am_ctx *c, const am_store *st, uint64_t n_new, const uint64_t *cap_hint, am_store **out) {
  AM_LOCK(c);
  const am_op_log &L = st->dev;
  if (n_new < L.n_keys) return AM_ERR_INVALID;
  if (!st->counter) {
    am_set_error("am_store_grow_keys: the store keeps no OpCounter column");
    return AM_ERR_INVALID;
  }
  const size_t o_end = am_round_up((n_new + 1) * 8, 256), o_idb = o_end + am_round_up(n_new * 8, 256);
  const size_t o_ctr = o_idb + am_round_up(n_new * 8, 256), o_type = o_ctr + am_round_up(n_new * 8, 256);
  const size_t o_flags = o_type + am_round_up(n_new, 256), total = o_flags + am_round_up(n_new, 256);
  void *scr = nullptr;
  if (int rc = am_dev_alloc(c, total, &scr)) return rc;
  char *b = (char *)scr;
  am_op_log view = L;
  view.n_keys = n_new;
  view.key_off = (uint64_t *)b, view.key_end = (uint64_t *)(b + o_end), view.key_id_base = (uint64_t *)(b + o_idb);
  view.key_type = (uint8_t *)(b + o_type), view.key_flags = (uint8_t *)(b + o_flags);
  view.key_tbase = nullptr, view.rec_key_off = nullptr, view.rec_key_end = nullptr, view.key_ngrp = nullptr;
  view.gmask = nullptr, view.zone_vc = nullptr, view.zone_gsum = nullptr, view.prec = nullptr;
  view.esc_rows = nullptr, view.lag_ct = nullptr, view.lag = nullptr, view.key_lag = nullptr;
  hipLaunchKernelGGL(k_grow_view, dim3(grid_threads(n_new + 1)), dim3(256), 0, c->stream, L,
                     (const uint64_t *)st->counter, n_new, (uint64_t *)view.key_off, (uint64_t *)view.key_end,
                     (uint64_t *)view.key_id_base, (uint64_t *)(b + o_ctr), (uint8_t *)view.key_type,
                     (uint8_t *)view.key_flags);
  int rc = hipGetLastError() == hipSuccess ? AM_OK : AM_ERR_HIP;
  if (!rc)
    rc = am_store_update_ex(c, view, (const uint64_t *)(b + o_ctr), nullptr, nullptr, nullptr, nullptr, nullptr, true,
                            cap_hint, out);
  (void)hipStreamSynchronize(c->stream);
  am_dev_release(c, scr);
  return rc;
}

extern "C" {

int am_store_reserve(am_ctx *c, const am_store *st, am_store **out) {
  if (!c || !st || !out) return AM_ERR_INVALID;
  AM_LOCK(c);
  AM_HIP(hipSetDevice(c->device));
  return am_store_update_ex(c, st->dev, st->counter, nullptr, nullptr, nullptr, nullptr, nullptr, true, nullptr, out);
}

int am_store_apply(am_ctx *c, am_store *st, uint64_t n_touched, const uint64_t *keys, const am_op_log *dev_new,
                   const uint8_t *prune_mask, const uint64_t *thr_vc, const uint32_t *thr_pres, uint8_t *gc_flags,
                   int *applied) {
  if (!c || !st || !applied || (n_touched && !keys) || (prune_mask && (!thr_vc || !thr_pres))) return AM_ERR_INVALID;
  AM_LOCK(c);
  *applied = 0;
  if (n_touched == 0) {
    *applied = 1;
    return AM_OK;
  }
  if (dev_new && (dev_new->n_dc != st->dev.n_dc || !dev_new->key_off || dev_new->n_keys != n_touched)) {
    am_set_error("am_store_apply: the new-op log must be CSR over the %llu touched keys with the store's n_dc",
                 (unsigned long long)n_touched);
    return AM_ERR_INVALID;
  }
  AM_HIP(hipSetDevice(c->device));
  // the key list comes from the caller: checked on the device (in range, distinct) inside the
  // apply, in the fit readback it already does; nothing is written when it fails
  return am_store_apply_ex(c, st, n_touched, keys, dev_new, prune_mask, thr_vc, thr_pres, gc_flags, nullptr, applied,
                           true);
}

}  // extern "C"
