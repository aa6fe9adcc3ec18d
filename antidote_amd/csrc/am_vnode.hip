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
#include <atomic>
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
  uint64_t rebuilds = 0;        // whole-store rebuilds (a key outgrew its room) ...
  uint64_t applies = 0;         // ... and in-place applies of touched keys
  std::atomic<int> in_flight{0};  // am_read_objects_submit tickets not yet finished
};

namespace {

// the reference's Length of key k
uint64_t ref_len(const am_vnode *v, uint64_t k) { return v->len[k] + v->quirk[k]; }

int swap_store(am_vnode *v, am_store *ns) {
  am_store_destroy(v->st);
  v->st = ns;
  return AM_OK;
}

// a device copy of a host key list (caching allocator; am_dev_release after use)
struct DevKeys {
  am_ctx *c;
  uint64_t *p = nullptr;
  explicit DevKeys(am_ctx *c_) : c(c_) {}
  int upload(const std::vector<uint64_t> &keys) {
    if (int rc = am_dev_alloc(c, keys.size() * 8 + 8, (void **)&p)) return rc;
    AM_HIP(hipMemcpyAsync(p, keys.data(), keys.size() * 8, hipMemcpyHostToDevice, c->stream));
    return AM_OK;
  }
  ~DevKeys() {
    if (p) {
      (void)hipStreamSynchronize(c->stream);
      am_dev_release(c, p);
    }
  }
};

// per-key op capacity for a rebuild (device [n], am_dev_release after use): room for the tuple's
// ListLen slots doubled once (snapshot_insert_gc/4's resize, src/materializer_vnode.erl:540-560:
// Length never exceeds ListLen, and a GC doubles ListLen when the tuple is nearly full), so a
// key outgrows its room only at its second doubling; keys without a tuple get the default room
struct CapHint {
  am_ctx *c;
  uint64_t *p = nullptr;
  explicit CapHint(am_ctx *c_) : c(c_) {}
  int upload(const am_vnode *v, uint64_t n) {
    std::vector<uint64_t> h(n, 0);
    for (uint64_t k = 0; k < n && k < v->list_len.size(); ++k)
      if (v->list_len[k]) h[k] = 2 * v->list_len[k] + 2;
    if (int rc = am_dev_alloc(c, n * 8 + 8, (void **)&p)) return rc;
    AM_HIP(hipMemcpyAsync(p, h.data(), n * 8, hipMemcpyHostToDevice, c->stream));
    AM_HIP(hipStreamSynchronize(c->stream));
    return AM_OK;
  }
  ~CapHint() {
    if (p) {
      (void)hipStreamSynchronize(c->stream);
      am_dev_release(c, p);
    }
  }
};

// NewListLen of snapshot_insert_gc/4 (src/materializer_vnode.erl:540-560) for key k
void resize_list_len(am_vnode *v, uint64_t k) {
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

// snapshot_insert_gc's op prune for `keys` (gc_mask set, thresholds on the device): in place
// (am_store_apply), or a whole-store rebuild when a key's room no longer fits; then
// NewListLen by the reference's resize rule
int prune(am_vnode *v, const std::vector<uint64_t> &keys) {
  const uint64_t m = keys.size();
  DevKeys dk(v->ctx);
  if (int rc = dk.upload(keys)) return rc;
  std::vector<uint64_t> nl(m);
  std::vector<uint8_t> fl(m);
  int applied = 0;
  int rc = am_store_apply_ex(v->ctx, v->st, m, dk.p, nullptr, v->gc_mask, v->thr_vc, v->thr_pres, v->gc_flags, nl.data(),
                          &applied);
  if (rc) return rc;
  if (applied) {
    ++v->applies;
    AM_HIP(hipMemcpyAsync(fl.data(), v->gc_flags, m, hipMemcpyDeviceToHost, v->ctx->stream));
    AM_HIP(hipStreamSynchronize(v->ctx->stream));
  } else {
    am_store *ns = nullptr;
    CapHint ch(v->ctx);
    if ((rc = ch.upload(v, v->n_keys))) return rc;
    rc = am_store_update_ex(v->ctx, v->st->dev, v->st->counter, nullptr, v->gc_mask, v->thr_vc, v->thr_pres,
                            v->gc_flags, true, ch.p, &ns);
    if (rc) return rc;
    swap_store(v, ns);
    ++v->rebuilds;
    rc = am_store_key_lens(v->ctx, v->st, m, dk.p, v->gc_flags, nl.data(), fl.data());
    if (rc) return rc;
  }
  for (uint64_t i = 0; i < m; ++i) {
    const uint64_t k = keys[i];
    v->len[k] = nl[i];
    v->quirk[k] = (fl[i] & AM_GC_PRUNED_ALL) ? 1 : 0;
    resize_list_len(v, k);
  }
  return AM_OK;
}

// a larger key space (keys [n_keys, new_n) have no tuple yet: ets:insert on their first op,
// src/materializer_vnode.erl:624-629): the store and snapshot cache grow, the device GC
// arrays are reallocated, the host mirrors extended
int grow_keys(am_vnode *v, uint64_t new_n) {
  if (new_n <= v->n_keys) return AM_OK;
  // every fallible step first (the new GC arrays, the grown store, the grown snapshot cache);
  // the vnode switches to them only when all succeeded, so a failure leaves it unchanged
  uint8_t *gm = nullptr, *gf = nullptr;
  uint64_t *tv = nullptr;
  uint32_t *tp = nullptr;
  am_store *ns = nullptr;
  int rc = am_dev_alloc(v->ctx, new_n + 16, (void **)&gm);
  if (!rc) rc = am_dev_alloc(v->ctx, new_n + 16, (void **)&gf);
  if (!rc) rc = am_dev_alloc(v->ctx, (size_t)v->n_dc * new_n * 8 + 16, (void **)&tv);
  if (!rc) rc = am_dev_alloc(v->ctx, new_n * 4 + 16, (void **)&tp);
  if (!rc && (hipMemsetAsync(gm, 0, new_n + 16, v->ctx->stream) != hipSuccess ||
              hipStreamSynchronize(v->ctx->stream) != hipSuccess)) {
    am_set_error("grow_keys: clearing the GC mask failed");
    rc = AM_ERR_HIP;
  }
  if (!rc) {
    CapHint ch(v->ctx);
    rc = ch.upload(v, new_n);
    if (!rc) rc = am_store_grow_keys(v->ctx, v->st, new_n, ch.p, &ns);
  }
  if (!rc) rc = am_snapcache_grow(v->sc, new_n);  // extra empty keys are harmless if a later step fails
  if (rc) {
    if (ns) am_store_destroy(ns);
    for (void *p : {(void *)gm, (void *)gf, (void *)tv, (void *)tp}) am_dev_release(v->ctx, p);
    return rc;
  }
  swap_store(v, ns);
  ++v->rebuilds;
  am_dev_release(v->ctx, v->gc_mask), am_dev_release(v->ctx, v->gc_flags);
  am_dev_release(v->ctx, v->thr_vc), am_dev_release(v->ctx, v->thr_pres);
  v->gc_mask = gm, v->gc_flags = gf, v->thr_vc = tv, v->thr_pres = tp;
  v->len.resize(new_n, 0), v->list_len.resize(new_n, 0), v->counter.resize(new_n, 0);
  v->quirk.resize(new_n, 0), v->type.resize(new_n, 0);
  v->n_keys = new_n;
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
  const uint64_t n = hb->n_reads;
  std::vector<uint8_t> sg(n, 0);
  if (should_gc) std::copy(should_gc, should_gc + n, sg.begin());
  int rc = am_run_host_batch(v->ctx, v->st, hb, hr, sg.data(), sg.size(), run_round, &a);
  if (rc) return rc;
  // the GC mask of the batch's keys only (keys past the vnode's are invalid reads)
  std::vector<uint64_t> keys;
  keys.reserve(n);
  for (uint64_t i = 0; i < n; ++i)
    if (hb->key[i] < v->n_keys) keys.push_back(hb->key[i]);
  if (keys.empty()) return AM_OK;
  DevKeys dk(v->ctx);
  if ((rc = dk.upload(keys))) return rc;
  std::vector<uint64_t> lens(keys.size());
  std::vector<uint8_t> mask(keys.size());
  rc = am_store_key_lens(v->ctx, v->st, keys.size(), dk.p, v->gc_mask, lens.data(), mask.data());
  if (rc) return rc;
  std::vector<uint64_t> gc;
  for (uint64_t i = 0; i < keys.size(); ++i)
    if (mask[i]) gc.push_back(keys[i]);
  return gc.empty() ? AM_OK : prune(v, gc);
}

// host op log holding the ops [beg_i, end_i) of source key src_i for every entry i of a list
// (same columns as src); key i of the slice is the list's entry i
struct HostSlice {
  am_op_log log{};
  std::vector<uint64_t> key_off, commit_time, snap_vc, op_txid, p0, p1, var_off, var_data;
  std::vector<uint8_t> key_type, key_flags, op_meta;
  std::vector<uint32_t> snap_pres;
  HostSlice(const am_op_log &s, const std::vector<uint64_t> &src, const std::vector<uint64_t> &beg,
            const std::vector<uint64_t> &end) {
    const uint64_t nk = src.size(), nd = s.n_dc, ss = s.snap_stride ? s.snap_stride : s.n_ops;
    key_off.assign(nk + 1, 0);
    for (uint64_t i = 0; i < nk; ++i) key_off[i + 1] = key_off[i] + (end[i] - beg[i]);
    const uint64_t n = key_off[nk];
    key_type.resize(nk);
    key_flags.resize(nk);
    for (uint64_t i = 0; i < nk; ++i) {
      key_type[i] = s.key_type[src[i]];
      key_flags[i] = s.key_flags ? s.key_flags[src[i]] : 0;
    }
    snap_vc.assign(nd * n, 0);
    if (s.var_off) var_off.assign(n + 1, 0);
    uint64_t q = 0;
    for (uint64_t i = 0; i < nk; ++i)
      for (uint64_t p = beg[i]; p < end[i]; ++p, ++q) {
        op_meta.push_back(s.op_meta[p]);
        commit_time.push_back(s.commit_time[p]);
        for (uint64_t d = 0; d < nd; ++d) snap_vc[d * n + q] = s.snap_vc[d * ss + p];
        if (s.snap_pres) snap_pres.push_back(s.snap_pres[p]);
        if (s.op_txid) op_txid.push_back(s.op_txid[p]);
        p0.push_back(s.p0[p]);
        p1.push_back(s.p1 ? s.p1[p] : 0);
        if (s.var_off) {
          for (uint64_t w = s.var_off[p]; w < s.var_off[p + 1]; ++w) var_data.push_back(s.var_data[w]);
          var_off[q + 1] = var_data.size();
        }
      }
    op_meta.push_back(0), commit_time.push_back(0), p0.push_back(0), p1.push_back(0);  // non-null when empty
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

// appends src's ops [beg_i, end_i) of source key src_i to vnode key keys_i (ids OpCounter +
// 1, ...): in place, or a whole-store rebuild with the new ops when a key outgrows its room
int append(am_vnode *v, const am_op_log &src, const std::vector<uint64_t> &keys, const std::vector<uint64_t> &srck,
           const std::vector<uint64_t> &beg, const std::vector<uint64_t> &end) {
  if (keys.empty()) return AM_OK;
  HostSlice hs(src, srck, beg, end);
  am_store *tmp = nullptr;
  int rc = am_store_create(v->ctx, &hs.log, &tmp);
  if (rc) return rc;
  DevKeys dk(v->ctx);
  int applied = 0;
  rc = dk.upload(keys);
  if (!rc) rc = am_store_apply_ex(v->ctx, v->st, keys.size(), dk.p, &tmp->dev, nullptr, nullptr, nullptr, nullptr, nullptr,
                               &applied);
  am_store_destroy(tmp);
  if (rc) return rc;
  if (applied) ++v->applies;
  if (!applied) {  // the new ops as CSR over every vnode key, one rebuild (every key's room regrown)
    std::vector<uint64_t> all_src(v->n_keys), all_beg(v->n_keys, 0), all_end(v->n_keys, 0);
    std::vector<uint8_t> tp(v->n_keys, AM_PN);
    for (uint64_t k = 0; k < v->n_keys; ++k) all_src[k] = k;
    am_op_log s2 = src;  // key types of untouched keys are never read (no ops)
    for (uint64_t i = 0; i < keys.size(); ++i) all_beg[keys[i]] = beg[i], all_end[keys[i]] = end[i];
    // HostSlice reads key_type / key_flags at the source key index: give it a vnode-indexed copy
    std::vector<uint8_t> kf(v->n_keys, 0);
    for (uint64_t i = 0; i < keys.size(); ++i) {
      tp[keys[i]] = src.key_type[srck[i]];
      kf[keys[i]] = src.key_flags ? src.key_flags[srck[i]] : 0;
    }
    s2.key_type = tp.data();
    s2.key_flags = src.key_flags ? kf.data() : nullptr;
    HostSlice all(s2, all_src, all_beg, all_end);
    am_store *t2 = nullptr;
    rc = am_store_create(v->ctx, &all.log, &t2);
    if (rc) return rc;
    am_store *ns = nullptr;
    CapHint ch(v->ctx);
    rc = ch.upload(v, v->n_keys);
    if (!rc)
      rc = am_store_update_ex(v->ctx, v->st->dev, v->st->counter, &t2->dev, nullptr, nullptr, nullptr, nullptr, true,
                              ch.p, &ns);
    am_store_destroy(t2);
    if (rc) return rc;
    swap_store(v, ns);
    ++v->rebuilds;
  }
  for (uint64_t i = 0; i < keys.size(); ++i) {
    v->len[keys[i]] += end[i] - beg[i];
    v->counter[keys[i]] += end[i] - beg[i];
  }
  return AM_OK;
}

// host result columns for n reads of an n_dc log with set capacity cap each
struct HostResult {
  am_read_result r{};
  std::vector<int32_t> status;
  std::vector<int64_t> nlo, v0;
  std::vector<uint64_t> last_ct, v1, set_off, set_a, set_b;
  std::vector<uint32_t> pres, count, set_len;
  std::vector<uint8_t> ign, newss, flags, vflag;
  HostResult(uint64_t n, uint32_t nd, uint64_t cap)
      : status(n), nlo(n), v0(n), last_ct(n * nd), v1(n), set_off(n + 1),
        set_a(n * cap + 1), set_b(n * cap + 1), pres(n), count(n), set_len(n), ign(n), newss(n), flags(n), vflag(n) {
    for (uint64_t i = 0; i <= n; ++i) set_off[i] = i * cap;
    r.status = status.data(), r.new_last_op = nlo.data(), r.last_ct = last_ct.data(), r.last_ct_pres = pres.data();
    r.last_ct_ignore = ign.data(), r.is_new_ss = newss.data(), r.count = count.data(), r.flags = flags.data();
    r.value.v0 = v0.data(), r.value.v1 = v1.data(), r.value.vflag = vflag.data();
    r.value.set_off = set_off.data(), r.value.set_len = set_len.data();
    r.value.set_a = set_a.data(), r.value.set_b = set_b.data();
  }
};

// op_insert_gc's GC reads: internal_read(Key, Type, Op.snapshot_time, ignore, [], true) for
// vnode key keys_i at the trigger op trig_i of the source log
int gc_reads(am_vnode *v, const am_op_log &src, std::vector<uint64_t> keys, std::vector<uint64_t> trig) {
  const uint64_t nd = v->n_dc, ss = src.snap_stride ? src.snap_stride : src.n_ops;
  const uint32_t all = nd >= 32 ? 0xFFFFFFFFu : ((1u << nd) - 1u);
  // the read's value is discarded; a read short of set capacity stored nothing and reruns
  for (uint64_t cap = 64; !keys.empty(); cap *= 4) {
    const uint64_t n = keys.size();
    std::vector<uint8_t> type(n), sg(n, 1);
    std::vector<uint64_t> vc(nd * n);
    std::vector<uint32_t> rp(n);
    for (uint64_t i = 0; i < n; ++i) {
      const uint64_t p = trig[i];
      type[i] = v->type[keys[i]];
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
    std::vector<uint64_t> again, again_t;
    for (uint64_t i = 0; i < n; ++i)
      if (hr.status[i] == AM_ERR_CAPACITY) again.push_back(keys[i]), again_t.push_back(trig[i]);
    keys.swap(again);
    trig.swap(again_t);
  }
  return AM_OK;
}

// op_insert_gc/3 for the ops [beg_i, end_i) of source key src_i into vnode key keys_i (keys
// distinct), each key oldest -> newest, in rounds: every key appends up to its next GC trigger
// (one in-place apply for all of them), the triggered keys' GC reads run as one batch (and
// prune in place), repeat.  Host work is O(touched keys) per round.
int insert_keys(am_vnode *v, const am_op_log &h, const std::vector<uint64_t> &keys, const std::vector<uint64_t> &srck,
                const std::vector<uint64_t> &beg, const std::vector<uint64_t> &end) {
  const uint64_t m = keys.size();
  std::vector<uint64_t> pos(beg);
  std::vector<uint8_t> pending(m, 0);  // the op at pos already ran its GC read
  std::vector<uint64_t> live;          // entries with ops left
  for (uint64_t i = 0; i < m; ++i)
    if (pos[i] < end[i]) live.push_back(i);
  while (!live.empty()) {
    // plan: each key appends up to (not including) its next trigger op
    std::vector<uint64_t> ak, asrc, abeg, aend, tk, tp, next;
    for (uint64_t i : live) {
      const uint64_t k = keys[i];
      if (!v->list_len[k]) v->list_len[k] = OPS_THRESHOLD, v->type[k] = h.key_type[srck[i]];  // ets:insert of a new tuple
      uint64_t p = pos[i], l = ref_len(v, k), c = v->counter[k];
      if (pending[i]) ++p, ++l, ++c;  // the trigger op goes in after its GC read
      uint64_t trig = ~0ull;
      for (; p < end[i]; ++p, ++l, ++c) {
        const uint64_t new_id = c + 1;
        if (l >= v->list_len[k] || new_id % OPS_THRESHOLD == 0) {
          trig = p;
          break;
        }
      }
      if (p > pos[i]) ak.push_back(k), asrc.push_back(srck[i]), abeg.push_back(pos[i]), aend.push_back(p);
      pos[i] = p;
      pending[i] = 0;
      if (trig != ~0ull) tk.push_back(k), tp.push_back(trig), pending[i] = 1;
      if (pos[i] < end[i]) next.push_back(i);
    }
    int rc = append(v, h, ak, asrc, abeg, aend);
    if (rc) return rc;
    if (!tk.empty() && (rc = gc_reads(v, h, tk, tp))) return rc;
    live.swap(next);
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
  am_ctx *c = v->ctx;
  while (v->in_flight.load()) std::this_thread::yield();  // submitted reads finish first
  std::lock_guard<std::recursive_mutex> lk(c->mu);       // and every call in progress
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
  if (!v || !h || h->n_keys < v->n_keys || h->n_dc != v->n_dc || !h->key_off || !h->key_type || !h->op_meta ||
      !h->commit_time || !h->p0 || (h->n_ops && !h->snap_vc)) {
    am_set_error("am_vnode_insert_host: the new ops must be a host log over (at least) the vnode's keys");
    return AM_ERR_INVALID;
  }
  AM_HIP(hipSetDevice(v->ctx->device));
  if (h->n_keys > v->n_keys)  // keys seen for the first time beyond the key space
    if (int rc = grow_keys(v, h->n_keys)) return rc;
  std::vector<uint64_t> keys, beg, end;
  for (uint64_t k = 0; k < v->n_keys; ++k)
    if (h->key_off[k + 1] > h->key_off[k]) keys.push_back(k), beg.push_back(h->key_off[k]), end.push_back(h->key_off[k + 1]);
  return insert_keys(v, *h, keys, keys, beg, end);
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
  AM_LOCK(v->ctx);
  if (st) *st = v->st;
  if (sc) *sc = v->sc;
  return AM_OK;
}

int am_vnode_stats(am_vnode *v, uint64_t *rebuilds, uint64_t *in_place) {
  if (!v) return AM_ERR_INVALID;
  AM_LOCK(v->ctx);
  if (rebuilds) *rebuilds = v->rebuilds;
  if (in_place) *in_place = v->applies;
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
  v->in_flight.fetch_add(1);
  t->th = std::thread([t, v, hr]() {
    t->rc = am_vnode_read_host(v, &t->b, nullptr, hr);
    v->in_flight.fetch_sub(1);
  });
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
