// am_vnode.hip -- one partition's materializer_vnode state on the device: the ops cache (an
// am_store, rebuilt by am_store_update) and the snapshot cache (am_snapcache), driven as the
// reference drives them (src/materializer_vnode.erl):
//   am_vnode_insert_host  op_insert_gc/3 (:622-647) for every new op, in order per key: the
//                         op gets NewId = OpCounter + 1; when Length >= ListLen or NewId rem
//                         OPS_THRESHOLD == 0 the insert first runs the GC read
//                         internal_read(Key, Type, Op.snapshot_time, ignore, [], true) and
//                         then appends.  load_ops/2 (:312-319) replays the log through the
//                         same call.
//   am_vnode_read_host    internal_read/7 (:371-376) for a batch, ShouldGC per read; a key
//                         read several times in one batch is served in batch order.
// A GC (snapshot_insert_gc/4, :515-563: the dict reached SNAPSHOT_THRESHOLD entries, or
// ShouldGC) truncates the key's snapshot dict to SNAPSHOT_MIN (am_snapcache), prunes its ops
// below their vectorclock:min (prune_ops/2 via am_store_update) and resizes ListLen by the
// reference's rule.  Batched: every key advances independently, so an insert batch runs in
// rounds -- append each key's ops up to its next GC trigger (one store rebuild for all
// keys), run the triggered keys' GC reads as one batch, prune them (one rebuild), repeat.
// The host keeps the per-key tuple header (Length, ListLen, OpCounter) the rounds plan with.
#include <algorithm>
#include <thread>

#include "am_internal.h"

int am_run_host_batch(am_ctx *c, const am_store *st, const am_read_batch *hb, am_read_result *hr,
                      const void *extra_host, size_t extra_bytes,
                      int (*run)(void *arg, const am_read_batch *db, am_read_result *dr, const void *extra_dev),
                      void *arg);  // am_host.hip

namespace {

constexpr uint64_t OPS_THRESHOLD = 50;   // src/materializer_vnode.erl:41
constexpr uint64_t RESIZE_THRESHOLD = 5; // :44

}  // namespace

struct am_vnode {
  am_ctx *ctx = nullptr;
  uint32_t n_dc = 0;
  uint64_t n_keys = 0;
  am_store *st = nullptr;
  am_snapcache *sc = nullptr;
  // the ops-cache tuple header per key: {Length, ListLen} and OpCounter; list_len 0 = no
  // tuple yet (ets:member false); quirk = prune_ops kept its element(FIRST_OP+Len)
  // placeholder (every op pruned): the reference's Length counts it, the device log holds 0
  std::vector<uint64_t> len, list_len, counter;
  std::vector<uint8_t> quirk, type;
  uint8_t *gc_mask = nullptr;   // device [n_keys]
  uint64_t *thr_vc = nullptr;   // device [n_dc][n_keys]
  uint32_t *thr_pres = nullptr; // device [n_keys]
  uint8_t *gc_flags = nullptr;  // device [n_keys]
};

namespace {

// the reference's Length of key k
uint64_t ref_len(const am_vnode *v, uint64_t k) { return v->len[k] + v->quirk[k]; }

// refreshes the Length mirror from the device log
int pull_lengths(am_vnode *v) {
  std::vector<uint64_t> ko(v->n_keys + 1);
  AM_HIP(hipMemcpyAsync(ko.data(), v->st->dev.key_off, (v->n_keys + 1) * 8, hipMemcpyDeviceToHost, v->ctx->stream));
  AM_HIP(hipStreamSynchronize(v->ctx->stream));
  for (uint64_t k = 0; k < v->n_keys; ++k) v->len[k] = ko[k + 1] - ko[k];
  return AM_OK;
}

int swap_store(am_vnode *v, am_store *ns) {
  am_store_destroy(v->st);
  v->st = ns;
  return AM_OK;
}

// snapshot_insert_gc's op prune for the keys in gc_mask (thresholds on the device), then
// NewListLen by the reference's resize rule
int prune(am_vnode *v, const std::vector<uint8_t> &mask) {
  am_store *ns = nullptr;
  int rc = am_store_update(v->ctx, v->st, nullptr, v->gc_mask, v->thr_vc, v->thr_pres, v->gc_flags, &ns);
  if (rc) return rc;
  swap_store(v, ns);
  std::vector<uint8_t> fl(v->n_keys);
  AM_HIP(hipMemcpyAsync(fl.data(), v->gc_flags, v->n_keys, hipMemcpyDeviceToHost, v->ctx->stream));
  AM_HIP(hipStreamSynchronize(v->ctx->stream));
  rc = pull_lengths(v);
  if (rc) return rc;
  for (uint64_t k = 0; k < v->n_keys; ++k) {
    if (!mask[k]) continue;
    v->quirk[k] = (fl[k] & AM_GC_PRUNED_ALL) ? 1 : 0;
    const uint64_t nl = ref_len(v, k), ll = v->list_len[k];
    uint64_t nll = ll;
    if (nl + RESIZE_THRESHOLD > ll) {  // NewLength > ListLen - RESIZE_THRESHOLD
      nll = ll * 2;
    } else {
      const uint64_t half = ll / 2;
      if (half > OPS_THRESHOLD && half > nl + RESIZE_THRESHOLD) nll = half;
    }
    v->list_len[k] = nll;
  }
  return AM_OK;
}

struct ReadArg {
  am_vnode *v;
};
int run_round(void *arg, const am_read_batch *db, am_read_result *dr, const void *extra_dev) {
  am_vnode *v = static_cast<ReadArg *>(arg)->v;
  return am_snapcache_read_gc(v->ctx, v->sc, &v->st->dev, db, (const uint8_t *)extra_dev, dr, v->gc_mask, v->thr_vc,
                              v->thr_pres);
}

// one round of reads over distinct keys (host arrays), then the GCs they triggered
int read_round(am_vnode *v, const am_read_batch *hb, const uint8_t *should_gc, am_read_result *hr) {
  ReadArg a{v};
  std::vector<uint8_t> sg(hb->n_reads, 0);
  if (should_gc) std::copy(should_gc, should_gc + hb->n_reads, sg.begin());
  int rc = am_run_host_batch(v->ctx, v->st, hb, hr, sg.data(), sg.size(), run_round, &a);
  if (rc) return rc;
  std::vector<uint8_t> mask(v->n_keys);
  AM_HIP(hipMemcpyAsync(mask.data(), v->gc_mask, v->n_keys, hipMemcpyDeviceToHost, v->ctx->stream));
  AM_HIP(hipStreamSynchronize(v->ctx->stream));
  if (std::any_of(mask.begin(), mask.end(), [](uint8_t x) { return x != 0; })) return prune(v, mask);
  return AM_OK;
}

// host op log holding, per key k, the ops [beg[k], end[k]) of src (same columns)
struct HostSlice {
  am_op_log log{};
  std::vector<uint64_t> key_off, commit_time, snap_vc, op_txid, p0, p1, var_off, var_data;
  std::vector<uint8_t> key_type, key_flags, op_meta;
  std::vector<uint32_t> snap_pres;
  HostSlice(const am_op_log &s, const std::vector<uint64_t> &beg, const std::vector<uint64_t> &end) {
    const uint64_t nk = s.n_keys, nd = s.n_dc, ss = s.snap_stride ? s.snap_stride : s.n_ops;
    key_off.assign(nk + 1, 0);
    for (uint64_t k = 0; k < nk; ++k) key_off[k + 1] = key_off[k] + (end[k] - beg[k]);
    const uint64_t n = key_off[nk];
    key_type.assign(s.key_type, s.key_type + nk);
    if (s.key_flags) key_flags.assign(s.key_flags, s.key_flags + nk);
    snap_vc.assign(nd * n, 0);
    if (s.var_off) var_off.assign(n + 1, 0);
    uint64_t q = 0;
    for (uint64_t k = 0; k < nk; ++k)
      for (uint64_t p = beg[k]; p < end[k]; ++p, ++q) {
        op_meta.push_back(s.op_meta[p]);
        commit_time.push_back(s.commit_time[p]);
        for (uint64_t d = 0; d < nd; ++d) snap_vc[d * n + q] = s.snap_vc[d * ss + p];
        if (s.snap_pres) snap_pres.push_back(s.snap_pres[p]);
        if (s.op_txid) op_txid.push_back(s.op_txid[p]);
        p0.push_back(s.p0[p]);
        p1.push_back(s.p1 ? s.p1[p] : 0);
        if (s.var_off) {
          for (uint64_t i = s.var_off[p]; i < s.var_off[p + 1]; ++i) var_data.push_back(s.var_data[i]);
          var_off[q + 1] = var_data.size();
        }
      }
    log.n_dc = s.n_dc;
    log.n_keys = nk;
    log.n_ops = n;
    log.n_var = var_data.size();
    log.snap_stride = n;
    log.key_off = key_off.data();
    log.key_type = key_type.data();
    log.key_flags = s.key_flags ? key_flags.data() : nullptr;
    log.op_meta = op_meta.data();
    log.commit_time = commit_time.data();
    log.snap_vc = snap_vc.data();
    log.snap_pres = s.snap_pres ? snap_pres.data() : nullptr;
    log.op_txid = s.op_txid ? op_txid.data() : nullptr;
    log.p0 = p0.data();
    log.p1 = p1.data();
    log.var_off = s.var_off ? var_off.data() : nullptr;
    log.var_data = s.var_off ? var_data.data() : nullptr;
  }
};

// appends src's ops [beg[k], end[k)) to every key (ids OpCounter + 1, ...)
int append(am_vnode *v, const am_op_log &src, const std::vector<uint64_t> &beg, const std::vector<uint64_t> &end) {
  HostSlice hs(src, beg, end);
  if (hs.log.n_ops == 0) return AM_OK;
  am_store *tmp = nullptr;
  int rc = am_store_create(v->ctx, &hs.log, &tmp);
  if (rc) return rc;
  am_store *ns = nullptr;
  rc = am_store_update(v->ctx, v->st, &tmp->dev, nullptr, nullptr, nullptr, nullptr, &ns);
  am_store_destroy(tmp);
  if (rc) return rc;
  swap_store(v, ns);
  for (uint64_t k = 0; k < v->n_keys; ++k) {
    v->len[k] += end[k] - beg[k];
    v->counter[k] += end[k] - beg[k];
  }
  return AM_OK;
}

// host result columns for n reads of an n_dc log with set capacity cap each
struct HostResult {
  am_read_result r{};
  std::vector<int32_t> status;
  std::vector<int64_t> nlo, v0, bc_p, bc_d;
  std::vector<uint64_t> last_ct, v1, set_off, set_a, set_b;
  std::vector<uint32_t> pres, count, set_len;
  std::vector<uint8_t> ign, newss, flags, vflag, bc_pp, bc_dp;
  HostResult(uint64_t n, uint32_t nd, uint64_t cap)
      : status(n), nlo(n), v0(n), bc_p(n * nd * nd), bc_d(n * nd), last_ct(n * nd), v1(n), set_off(n + 1),
        set_a(n * cap + 1), set_b(n * cap + 1), pres(n), count(n), set_len(n), ign(n), newss(n), flags(n), vflag(n),
        bc_pp(n * nd * nd), bc_dp(n * nd) {
    for (uint64_t i = 0; i <= n; ++i) set_off[i] = i * cap;
    r.status = status.data(), r.new_last_op = nlo.data(), r.last_ct = last_ct.data(), r.last_ct_pres = pres.data();
    r.last_ct_ignore = ign.data(), r.is_new_ss = newss.data(), r.count = count.data(), r.flags = flags.data();
    r.value.v0 = v0.data(), r.value.v1 = v1.data(), r.value.vflag = vflag.data();
    r.value.set_off = set_off.data(), r.value.set_len = set_len.data();
    r.value.set_a = set_a.data(), r.value.set_b = set_b.data();
    r.value.bc_p = bc_p.data(), r.value.bc_p_pres = bc_pp.data(), r.value.bc_d = bc_d.data(),
    r.value.bc_d_pres = bc_dp.data();
  }
};

// op_insert_gc's GC reads: internal_read(Key, Type, Op.snapshot_time, ignore, [], true) for
// the trigger op trig[k] of every key with one (~0 = none)
int gc_reads(am_vnode *v, const am_op_log &src, const std::vector<uint64_t> &trig) {
  std::vector<uint64_t> keys;
  for (uint64_t k = 0; k < v->n_keys; ++k)
    if (trig[k] != ~0ull) keys.push_back(k);
  const uint64_t nd = v->n_dc, ss = src.snap_stride ? src.snap_stride : src.n_ops;
  const uint32_t all = nd >= 32 ? 0xFFFFFFFFu : ((1u << nd) - 1u);
  // the read's value is discarded; a read short of set capacity stored nothing and reruns
  for (uint64_t cap = 64; !keys.empty(); cap *= 4) {
    const uint64_t n = keys.size();
    std::vector<uint8_t> type(n), sg(n, 1);
    std::vector<uint64_t> vc(nd * n);
    std::vector<uint32_t> rp(n);
    for (uint64_t i = 0; i < n; ++i) {
      const uint64_t k = keys[i], p = trig[k];
      type[i] = src.key_type[k];
      rp[i] = src.snap_pres ? (src.snap_pres[p] & all) : all;
      for (uint64_t d = 0; d < nd; ++d) vc[d * n + i] = ((rp[i] >> d) & 1u) ? src.snap_vc[d * ss + p] : 0;
    }
    am_read_batch b{};
    b.n_reads = n;
    b.per_read_clock = 1;
    b.key = keys.data();
    b.type = type.data();
    b.read_vc = vc.data();
    b.read_pres = rp.data();
    HostResult hr(n, v->n_dc, cap);
    int rc = read_round(v, &b, sg.data(), &hr.r);
    if (rc) return rc;
    std::vector<uint64_t> again;
    for (uint64_t i = 0; i < n; ++i)
      if (hr.status[i] == AM_ERR_CAPACITY) again.push_back(keys[i]);
    keys.swap(again);
  }
  return AM_OK;
}

}  // namespace

extern "C" {

int am_vnode_create(am_ctx *ctx, uint32_t n_dc, uint64_t n_keys, am_vnode **out) {
  if (!ctx || !out || n_dc == 0 || n_dc > AM_MAX_DC || n_keys == 0) return AM_ERR_INVALID;
  AM_HIP(hipSetDevice(ctx->device));
  am_vnode *v = new am_vnode();
  v->ctx = ctx, v->n_dc = n_dc, v->n_keys = n_keys;
  v->len.assign(n_keys, 0), v->list_len.assign(n_keys, 0), v->counter.assign(n_keys, 0);
  v->quirk.assign(n_keys, 0), v->type.assign(n_keys, 0);
  // the empty ops cache
  std::vector<uint64_t> ko(n_keys + 1, 0), ct(1, 0), p0(1, 0), vo(1, 0);
  std::vector<uint8_t> kt(n_keys, AM_PN), om(1, 0);
  am_op_log h{};
  h.n_dc = n_dc, h.n_keys = n_keys, h.n_ops = 0;
  h.key_off = ko.data(), h.key_type = kt.data(), h.op_meta = om.data(), h.commit_time = ct.data(), h.p0 = p0.data();
  h.p1 = p0.data(), h.var_off = vo.data();
  int rc = am_store_create(ctx, &h, &v->st);
  if (!rc) rc = am_snapcache_create(ctx, n_dc, n_keys, &v->sc);
  if (!rc) rc = am_dev_alloc(ctx, n_keys + 16, (void **)&v->gc_mask);
  if (!rc) rc = am_dev_alloc(ctx, n_keys + 16, (void **)&v->gc_flags);
  if (!rc) rc = am_dev_alloc(ctx, (size_t)n_dc * n_keys * 8 + 16, (void **)&v->thr_vc);
  if (!rc) rc = am_dev_alloc(ctx, n_keys * 4 + 16, (void **)&v->thr_pres);
  if (rc) {
    am_vnode_destroy(v);
    return rc;
  }
  *out = v;
  return AM_OK;
}

int am_vnode_destroy(am_vnode *v) {
  if (!v) return AM_OK;
  if (v->st) am_store_destroy(v->st);
  if (v->sc) am_snapcache_destroy(v->sc);
  if (v->gc_mask) am_dev_free(v->ctx, v->gc_mask);
  if (v->gc_flags) am_dev_free(v->ctx, v->gc_flags);
  if (v->thr_vc) am_dev_free(v->ctx, v->thr_vc);
  if (v->thr_pres) am_dev_free(v->ctx, v->thr_pres);
  delete v;
  return AM_OK;
}

int am_vnode_insert_host(am_vnode *v, const am_op_log *h) {
  if (!v) return AM_ERR_INVALID;
  AM_LOCK(v->ctx);
  if (!v || !h || h->n_keys != v->n_keys || h->n_dc != v->n_dc || !h->key_off || !h->key_type || !h->op_meta ||
      !h->commit_time || !h->p0 || (h->n_ops && !h->snap_vc)) {
    am_set_error("am_vnode_insert_host: the new ops must be a host log over the vnode's keys");
    return AM_ERR_INVALID;
  }
  AM_HIP(hipSetDevice(v->ctx->device));
  const uint64_t nk = v->n_keys;
  std::vector<uint64_t> pos(nk), end(nk);
  std::vector<uint8_t> pending(nk, 0);  // the op at pos already ran its GC read
  for (uint64_t k = 0; k < nk; ++k) pos[k] = h->key_off[k], end[k] = h->key_off[k + 1];
  for (;;) {
    // plan: each key appends up to (not including) its next trigger op
    std::vector<uint64_t> seg_end(nk), trig(nk, ~0ull);
    bool any = false;
    for (uint64_t k = 0; k < nk; ++k) {
      if (pos[k] == end[k]) {
        seg_end[k] = pos[k];
        continue;
      }
      any = true;
      if (!v->list_len[k]) v->list_len[k] = OPS_THRESHOLD, v->type[k] = h->key_type[k];  // ets:insert of a new tuple
      uint64_t p = pos[k], l = ref_len(v, k), c = v->counter[k];
      if (pending[k]) ++p, ++l, ++c;  // the trigger op goes in after its GC read
      for (; p < end[k]; ++p, ++l, ++c) {
        const uint64_t new_id = c + 1;
        if (l >= v->list_len[k] || new_id % OPS_THRESHOLD == 0) {
          trig[k] = p;
          break;
        }
      }
      seg_end[k] = p;
    }
    if (!any) break;
    int rc = append(v, *h, pos, seg_end);
    if (rc) return rc;
    for (uint64_t k = 0; k < nk; ++k) pos[k] = seg_end[k], pending[k] = 0;
    rc = gc_reads(v, *h, trig);
    if (rc) return rc;
    for (uint64_t k = 0; k < nk; ++k)
      if (trig[k] != ~0ull) pending[k] = 1;
  }
  return AM_OK;
}

int am_vnode_read_host(am_vnode *v, const am_read_batch *hb, const uint8_t *should_gc, am_read_result *hr) {
  if (!v) return AM_ERR_INVALID;
  AM_LOCK(v->ctx);
  if (!v || !hb || !hr || !hb->key || !hb->type || !hb->read_vc || !hb->read_pres) return AM_ERR_INVALID;
  AM_HIP(hipSetDevice(v->ctx->device));
  const uint64_t n = hb->n_reads, nd = v->n_dc;
  if (n == 0) return AM_OK;
  // occurrence rank of every read among the reads of its key: round j serves rank j
  std::vector<uint32_t> occ(n);
  {
    std::vector<uint64_t> idx(n);
    for (uint64_t i = 0; i < n; ++i) idx[i] = i;
    std::stable_sort(idx.begin(), idx.end(), [&](uint64_t a, uint64_t b) { return hb->key[a] < hb->key[b]; });
    for (uint64_t j = 0; j < n; ++j) occ[idx[j]] = (j && hb->key[idx[j]] == hb->key[idx[j - 1]]) ? occ[idx[j - 1]] + 1 : 0;
  }
  const uint32_t rounds = 1 + *std::max_element(occ.begin(), occ.end());
  if (rounds == 1) return read_round(v, hb, should_gc, hr);
  const uint64_t np = nd * nd;
  for (uint32_t j = 0; j < rounds; ++j) {
    std::vector<uint64_t> sel;
    for (uint64_t i = 0; i < n; ++i)
      if (occ[i] == j) sel.push_back(i);
    const uint64_t m = sel.size();
    // the round's sub-batch (cache-served reads ignore the batch's base members)
    std::vector<uint64_t> key(m), vc(nd * (hb->per_read_clock ? m : 1)), txid(m), so(m + 1, 0);
    std::vector<uint8_t> type(m), txv(m, 1), sg(m, 0);
    std::vector<uint32_t> rp(hb->per_read_clock ? m : 1);
    for (uint64_t q = 0; q < m; ++q) {
      const uint64_t i = sel[q];
      key[q] = hb->key[i], type[q] = hb->type[i];
      if (hb->txid) txid[q] = hb->txid[i], txv[q] = hb->txid_valid ? hb->txid_valid[i] : 1;
      if (should_gc) sg[q] = should_gc[i];
      if (hb->per_read_clock) {
        rp[q] = hb->read_pres[i];
        for (uint64_t d = 0; d < nd; ++d) vc[d * m + q] = hb->read_vc[d * n + i];
      }
      so[q + 1] = so[q] + (hr->value.set_off ? hr->value.set_off[i + 1] - hr->value.set_off[i] : 0);
    }
    if (!hb->per_read_clock) {
      rp[0] = hb->read_pres[0];
      for (uint64_t d = 0; d < nd; ++d) vc[d] = hb->read_vc[d];
    }
    am_read_batch b{};
    b.n_reads = m, b.per_read_clock = hb->per_read_clock, b.type_hint = hb->type_hint;
    b.key = key.data(), b.type = type.data(), b.read_vc = vc.data(), b.read_pres = rp.data();
    if (hb->txid) b.txid = txid.data(), b.txid_valid = txv.data();
    HostResult res(m, v->n_dc, 0);
    res.set_off = so;
    res.set_a.assign(so[m] + 1, 0), res.set_b.assign(so[m] + 1, 0);
    res.r.value.set_off = res.set_off.data(), res.r.value.set_a = res.set_a.data(), res.r.value.set_b = res.set_b.data();
    int rc = read_round(v, &b, sg.data(), &res.r);
    if (rc) return rc;
    for (uint64_t q = 0; q < m; ++q) {  // scatter to the caller's columns
      const uint64_t i = sel[q];
      hr->status[i] = res.status[q], hr->new_last_op[i] = res.nlo[q], hr->last_ct_pres[i] = res.pres[q];
      hr->last_ct_ignore[i] = res.ign[q], hr->is_new_ss[i] = res.newss[q], hr->count[i] = res.count[q];
      hr->flags[i] = res.flags[q];
      for (uint64_t d = 0; d < nd; ++d) hr->last_ct[d * n + i] = res.last_ct[d * m + q];
      if (hr->value.v0) hr->value.v0[i] = res.v0[q];
      if (hr->value.v1) hr->value.v1[i] = res.v1[q];
      if (hr->value.vflag) hr->value.vflag[i] = res.vflag[q];
      if (hr->value.set_len) {
        hr->value.set_len[i] = res.set_len[q];
        for (uint64_t x = 0; x < res.set_len[q] && x < so[q + 1] - so[q]; ++x) {
          hr->value.set_a[hr->value.set_off[i] + x] = res.set_a[so[q] + x];
          hr->value.set_b[hr->value.set_off[i] + x] = res.set_b[so[q] + x];
        }
      }
      if (hr->value.bc_p)
        for (uint64_t s = 0; s < np; ++s)
          hr->value.bc_p[i * np + s] = res.bc_p[q * np + s], hr->value.bc_p_pres[i * np + s] = res.bc_pp[q * np + s];
      if (hr->value.bc_d)
        for (uint64_t s = 0; s < nd; ++s)
          hr->value.bc_d[i * nd + s] = res.bc_d[q * nd + s], hr->value.bc_d_pres[i * nd + s] = res.bc_dp[q * nd + s];
    }
  }
  return AM_OK;
}

int am_vnode_relabel(am_vnode *v, const uint64_t *old_labels, const uint64_t *new_labels, uint64_t n) {
  if (!v) return AM_ERR_INVALID;
  AM_LOCK(v->ctx);
  int rc = am_store_relabel(v->ctx, v->st, old_labels, new_labels, n);
  if (!rc) rc = am_snapcache_relabel(v->ctx, v->sc, v->st->dev.key_type, old_labels, new_labels, n);
  return rc;
}

int am_vnode_parts(am_vnode *v, am_store **st, am_snapcache **sc) {
  if (!v) return AM_ERR_INVALID;
  if (st) *st = v->st;
  if (sc) *sc = v->sc;
  return AM_OK;
}

int am_vnode_key_info(am_vnode *v, uint64_t key, uint64_t *length, uint64_t *list_len, uint64_t *op_counter) {
  if (!v) return AM_ERR_INVALID;
  AM_LOCK(v->ctx);
  if (!v || key >= v->n_keys) return AM_ERR_INVALID;
  if (length) *length = ref_len(v, key);
  if (list_len) *list_len = v->list_len[key];
  if (op_counter) *op_counter = v->counter[key];
  return AM_OK;
}

}  // extern "C"

// ---- read_objects over a node's partitions: one vnode whose key space concatenates them
struct am_ticket {
  std::thread th;
  int rc = AM_OK;
  am_read_batch b{};
  std::vector<uint64_t> key;
};

namespace {

// the requests' vnode keys (part_key_base[part] + local key); an out-of-range request gets a
// key past the vnode's, which the read reports as AM_ERR_INVALID
int objects_keys(am_vnode *v, uint32_t n_parts, const uint64_t *base, const uint32_t *part, const am_read_batch *hb,
                 std::vector<uint64_t> &key) {
  if (!v || !base || !hb || (hb->n_reads && (!part || !hb->key))) return AM_ERR_INVALID;
  if (base[n_parts] > v->n_keys) {
    am_set_error("am_read_objects: partition key ranges exceed the vnode's keys");
    return AM_ERR_INVALID;
  }
  key.resize(hb->n_reads);
  for (uint64_t i = 0; i < hb->n_reads; ++i) {
    const uint32_t p = part[i];
    const bool ok = p < n_parts && base[p] <= base[p + 1] && hb->key[i] < base[p + 1] - base[p];
    key[i] = ok ? base[p] + hb->key[i] : ~0ull;
  }
  return AM_OK;
}

}  // namespace

extern "C" {

int am_read_objects_host(am_vnode *v, uint32_t n_parts, const uint64_t *part_key_base, const uint32_t *part,
                         const am_read_batch *hb, am_read_result *hr) {
  std::vector<uint64_t> key;
  if (int rc = objects_keys(v, n_parts, part_key_base, part, hb, key)) return rc;
  am_read_batch b = *hb;
  b.key = key.data();
  return am_vnode_read_host(v, &b, nullptr, hr);
}

int am_read_objects_submit(am_vnode *v, uint32_t n_parts, const uint64_t *part_key_base, const uint32_t *part,
                           const am_read_batch *hb, am_read_result *hr, am_ticket **out) {
  if (!out) return AM_ERR_INVALID;
  am_ticket *t = new am_ticket();
  if (int rc = objects_keys(v, n_parts, part_key_base, part, hb, t->key)) {
    delete t;
    return rc;
  }
  t->b = *hb;
  t->b.key = t->key.data();
  t->th = std::thread([t, v, hr]() { t->rc = am_vnode_read_host(v, &t->b, nullptr, hr); });
  *out = t;
  return AM_OK;
}

int am_ticket_wait(am_ticket *t) {
  if (!t) return AM_ERR_INVALID;
  if (t->th.joinable()) t->th.join();
  const int rc = t->rc;
  delete t;
  return rc;
}

}  // extern "C"
