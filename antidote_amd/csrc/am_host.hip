// am_host.hip -- am_materialize_host: the blocking, host-memory form of the hot
// path that a (dirty) Erlang NIF calls per batch of reads.  Stages the batch
// into one device arena, runs am_materialize on the store's resident log and
// copies the result columns back.
#include <cstring>
#include <functional>
#include <vector>

#include "am_internal.h"

namespace {

struct Arena {
  std::vector<std::pair<const void *, size_t>> in;  // (host src, bytes) in order
  size_t bytes = 0;
  size_t add(size_t n) {
    size_t off = bytes;
    bytes += (n + 255) & ~(size_t)255;
    return off;
  }
};

}  // namespace

// Stages a host batch into one device arena, runs `run` on the device batch/result and
// copies the result columns back.
static int run_host(am_ctx *c, const am_store *st, const am_read_batch *hb, am_read_result *hr,
                    const std::function<int(const am_read_batch *, am_read_result *, const void *)> &run,
                    const void *extra_host = nullptr, size_t extra_bytes = 0) {
  if (!c || !st || !hb || !hr || !hb->key || !hb->type || !hb->read_vc || !hb->read_pres) return AM_ERR_INVALID;
  const uint64_t n = hb->n_reads;
  if (n == 0) return AM_OK;
  const uint32_t nd = st->dev.n_dc;
  const uint64_t nclk = hb->per_read_clock ? n : 1;
  const uint64_t nset_in = hb->base.set_off ? hb->base.set_off[n] : 0;
  const uint64_t nset_out = hr->value.set_off ? hr->value.set_off[n] : 0;

  struct In {
    const void *h;
    size_t bytes;
    const void **dptr;
  };
  struct Out {
    void *h;
    size_t bytes;
    void **dptr;
  };
  am_read_batch db = *hb;
  am_read_result dr = *hr;
  std::vector<In> ins;
  std::vector<Out> outs;
  auto in = [&](const void *h, size_t bytes, const void **slot) {
    if (h) ins.push_back({h, bytes, slot});
  };
  auto out = [&](void *h, size_t bytes, void **slot) {
    if (h) outs.push_back({h, bytes, slot});
  };
  in(hb->key, n * 8, (const void **)&db.key);
  in(hb->type, n, (const void **)&db.type);
  in(hb->read_vc, nclk * nd * 8, (const void **)&db.read_vc);
  in(hb->read_pres, nclk * 4, (const void **)&db.read_pres);
  in(hb->txid, n * 8, (const void **)&db.txid);
  in(hb->txid_valid, n, (const void **)&db.txid_valid);
  in(hb->base_ignore, n, (const void **)&db.base_ignore);
  in(hb->base_vc, n * nd * 8, (const void **)&db.base_vc);
  in(hb->base_pres, n * 4, (const void **)&db.base_pres);
  in(hb->base_last_op, n * 8, (const void **)&db.base_last_op);
  in(hb->base.v0, n * 8, (const void **)&db.base.v0);
  in(hb->base.v1, n * 8, (const void **)&db.base.v1);
  in(hb->base.vflag, n, (const void **)&db.base.vflag);
  in(hb->base.set_off, (n + 1) * 8, (const void **)&db.base.set_off);
  in(hb->base.set_len, n * 4, (const void **)&db.base.set_len);
  in(hb->base.set_a, nset_in * 8, (const void **)&db.base.set_a);
  in(hb->base.set_b, nset_in * 8, (const void **)&db.base.set_b);
  in(hr->value.set_off, (n + 1) * 8, (const void **)&dr.value.set_off);
  const void *extra_dev = nullptr;
  in(extra_host, extra_bytes, &extra_dev);

  out(hr->status, n * 4, (void **)&dr.status);
  out(hr->new_last_op, n * 8, (void **)&dr.new_last_op);
  out(hr->last_ct, n * nd * 8, (void **)&dr.last_ct);
  out(hr->last_ct_pres, n * 4, (void **)&dr.last_ct_pres);
  out(hr->last_ct_ignore, n, (void **)&dr.last_ct_ignore);
  out(hr->is_new_ss, n, (void **)&dr.is_new_ss);
  out(hr->count, n * 4, (void **)&dr.count);
  out(hr->flags, n, (void **)&dr.flags);
  out(hr->value.v0, n * 8, (void **)&dr.value.v0);
  out(hr->value.v1, n * 8, (void **)&dr.value.v1);
  out(hr->value.vflag, n, (void **)&dr.value.vflag);
  out(hr->value.set_len, n * 4, (void **)&dr.value.set_len);
  out(hr->value.set_a, nset_out * 8, (void **)&dr.value.set_a);
  out(hr->value.set_b, nset_out * 8, (void **)&dr.value.set_b);
  if (!hr->status || !hr->new_last_op || !hr->last_ct || !hr->last_ct_pres || !hr->last_ct_ignore || !hr->is_new_ss ||
      !hr->count || !hr->flags) {
    am_set_error("host batch: every result column is required");
    return AM_ERR_INVALID;
  }

  size_t total = 0;
  std::vector<size_t> in_off(ins.size()), out_off(outs.size());
  for (size_t i = 0; i < ins.size(); ++i) {
    in_off[i] = total;
    total += (ins[i].bytes + 255) & ~(size_t)255;
  }
  for (size_t i = 0; i < outs.size(); ++i) {
    out_off[i] = total;
    total += (outs[i].bytes + 255) & ~(size_t)255;
  }
  AM_HIP(hipSetDevice(c->device));
  char *arena = nullptr;
  int rc = am_dev_alloc(c, total ? total : 256, (void **)&arena);
  if (rc) return rc;
  hipError_t e = hipSuccess;
  for (size_t i = 0; i < ins.size() && e == hipSuccess; ++i) {
    e = hipMemcpyAsync(arena + in_off[i], ins[i].h, ins[i].bytes, hipMemcpyHostToDevice, c->stream);
    *ins[i].dptr = arena + in_off[i];
  }
  for (size_t i = 0; i < outs.size() && e == hipSuccess; ++i) {
    e = hipMemsetAsync(arena + out_off[i], 0, outs[i].bytes, c->stream);
    *outs[i].dptr = arena + out_off[i];
  }
  if (e == hipSuccess) {
    rc = run(&db, &dr, extra_dev);
    for (size_t i = 0; i < outs.size() && e == hipSuccess && !rc; ++i)
      e = hipMemcpyAsync(outs[i].h, arena + out_off[i], outs[i].bytes, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  }
  am_dev_release(c, arena);  // stream-ordered reuse by the next host batch
  if (e != hipSuccess) {
    am_set_error("host batch: %s", hipGetErrorString(e));
    return AM_ERR_HIP;
  }
  return rc;
}

extern "C" int am_materialize_host(am_ctx *c, const am_store *st, const am_read_batch *hb, am_read_result *hr) {
  if (!c) return AM_ERR_INVALID;
  AM_LOCK(c);
  if (!st) return AM_ERR_INVALID;
  return run_host(c, st, hb, hr, [&](const am_read_batch *db, am_read_result *dr, const void *) {
    return am_launch_materialize(c, &st->dev, db, dr);
  });
}

extern "C" int am_snapcache_read_host(am_ctx *c, am_snapcache *sc, const am_store *st, const am_read_batch *hb,
                                      am_read_result *hr) {
  if (!st || !sc) return AM_ERR_INVALID;
  if (!c) return AM_ERR_INVALID;
  AM_LOCK(c);
  return run_host(c, st, hb, hr, [&](const am_read_batch *db, am_read_result *dr, const void *) {
    return am_snapcache_read(c, sc, &st->dev, db, dr);
  });
}

// run_host for internal callers: `run` also gets extra_host staged to the device (am_vnode.hip)
int am_run_host_batch(am_ctx *c, const am_store *st, const am_read_batch *hb, am_read_result *hr,
                      const void *extra_host, size_t extra_bytes,
                      int (*run)(void *arg, const am_read_batch *db, am_read_result *dr, const void *extra_dev),
                      void *arg) {
  return run_host(
      c, st, hb, hr,
      [&](const am_read_batch *db, am_read_result *dr, const void *extra_dev) { return run(arg, db, dr, extra_dev); },
      extra_host, extra_bytes);
}
