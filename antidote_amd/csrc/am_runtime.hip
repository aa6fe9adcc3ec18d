// am_runtime.hip -- context, device memory, op-log stores, timers and the C ABI
// entry points of libantidote_mat.so (declared in include/antidote_mat.h).
#include <cstdlib>
#include <cstring>
#include <string>

#include "am_internal.h"

static thread_local char g_err[512] = {0};

void am_set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

extern "C" {

int am_abi_version(void) { return AM_ABI_VERSION; }
const char *am_last_error(void) { return g_err; }

int am_ctx_open(int device, am_ctx **out) {
  if (!out) return AM_ERR_INVALID;
  int ndev = 0;
  AM_HIP(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) {
    am_set_error("device %d out of range (%d devices)", device, ndev);
    return AM_ERR_INVALID;
  }
  AM_HIP(hipSetDevice(device));
  am_ctx *c = new am_ctx();
  c->device = device;
  hipDeviceProp_t prop;
  AM_HIP(hipGetDeviceProperties(&prop, device));
  c->n_cu = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  AM_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  AM_HIP(hipEventCreate(&c->ev0));
  AM_HIP(hipEventCreate(&c->ev1));
  AM_HIP(hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming));
  AM_HIP(hipMalloc((void **)&c->stats, 8 * sizeof(uint64_t)));
  AM_HIP(hipMemsetAsync(c->stats, 0, 8 * sizeof(uint64_t), c->stream));
  *out = c;
  return AM_OK;
}

int am_ctx_close(am_ctx *c) {
  if (!c) return AM_OK;
  AM_HIP(hipSetDevice(c->device));
  for (am_ctx *&s : c->sub)
    if (s) (void)am_ctx_close(s), s = nullptr;
  AM_HIP(hipStreamSynchronize(c->stream));
  for (void *&p : c->scratch)
    if (p) (void)hipFree(p), p = nullptr;
  for (auto &kv : c->free_blocks) (void)hipFree(kv.second);
  c->free_blocks.clear();
  if (c->pinned) (void)hipHostFree(c->pinned), c->pinned = nullptr;
  if (c->stats && !c->is_sub) (void)hipFree(c->stats);
  c->stats = nullptr;
  (void)hipEventDestroy(c->ev0);
  (void)hipEventDestroy(c->ev1);
  if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
  (void)hipStreamDestroy(c->stream);
  delete c;
  return AM_OK;
}

void *am_ctx_stream(am_ctx *c) { return c ? (void *)c->stream : nullptr; }

int am_ctx_sync(am_ctx *c) {
  if (!c) return AM_ERR_INVALID;
  AM_LOCK(c);
  AM_HIP(hipStreamSynchronize(c->stream));
  return AM_OK;
}

int am_ctx_stat(am_ctx *c, int which, uint64_t *value, int reset) {
  if (!c || !value || which < AM_STAT_OPS_SKIPPED || which > AM_STAT_GSUM_WORDS) return AM_ERR_INVALID;
  AM_LOCK(c);
  AM_HIP(hipSetDevice(c->device));
  if (int rc = am_ctx_fetch(c, c->stats + which, 1, value)) return rc;
  if (reset) AM_HIP(hipMemsetAsync(c->stats + which, 0, sizeof(uint64_t), c->stream));
  return AM_OK;
}

int am_timer_start(am_ctx *c) {
  if (!c) return AM_ERR_INVALID;
  AM_LOCK(c);
  AM_HIP(hipEventRecord(c->ev0, c->stream));
  return AM_OK;
}

int am_timer_stop(am_ctx *c, float *ms) {
  if (!c || !ms) return AM_ERR_INVALID;
  AM_LOCK(c);
  AM_HIP(hipEventRecord(c->ev1, c->stream));
  AM_HIP(hipEventSynchronize(c->ev1));
  AM_HIP(hipEventElapsedTime(ms, c->ev0, c->ev1));
  return AM_OK;
}

}  // extern "C"

am_ctx *am_ctx_sub(am_ctx *c, int i) {
  if (c->sub[i]) return c->sub[i];
  am_ctx *s = new am_ctx();
  s->device = c->device;
  s->n_cu = c->n_cu;
  s->is_sub = true;
  s->stats = c->stats;
  if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&s->ev0, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&s->ev1, hipEventDisableTiming) != hipSuccess) {
    am_set_error("sub-context stream / events: %s", hipGetErrorString(hipGetLastError()));
    if (s->stream) (void)hipStreamDestroy(s->stream);
    if (s->ev0) (void)hipEventDestroy(s->ev0);
    delete s;
    return nullptr;
  }
  return c->sub[i] = s;
}

int am_ctx_scratch(am_ctx *c, int slot, size_t bytes, void **out) {
  if (!c || slot < 0 || slot >= AM_N_SCR || !out) return AM_ERR_INVALID;
  if (bytes == 0) bytes = 256;
  if (c->scratch_bytes[slot] < bytes) {
    if (c->scratch[slot]) {
      AM_HIP(hipStreamSynchronize(c->stream));
      AM_HIP(hipFree(c->scratch[slot]));
      c->scratch[slot] = nullptr;
      c->scratch_bytes[slot] = 0;
    }
    const size_t want = bytes + bytes / 4;  // headroom against regrowth
    void *p = nullptr;
    const hipError_t e = hipMalloc(&p, want);
    if (e != hipSuccess) {
      am_set_error("scratch hipMalloc(%zu): %s", want, hipGetErrorString(e));
      return AM_ERR_NOMEM;
    }
    c->scratch[slot] = p;
    c->scratch_bytes[slot] = want;
  }
  *out = c->scratch[slot];
  return AM_OK;
}

int am_ctx_fetch(am_ctx *c, const void *dev, uint32_t n, uint64_t *host) {
  AM_LOCK(c);
  if (n > 64) return AM_ERR_INVALID;
  if (!c->pinned) AM_HIP(hipHostMalloc((void **)&c->pinned, 64 * sizeof(uint64_t), hipHostMallocDefault));
  AM_HIP(hipMemcpyAsync(c->pinned, dev, n * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
  AM_HIP(hipStreamSynchronize(c->stream));
  memcpy(host, c->pinned, n * sizeof(uint64_t));
  return AM_OK;
}

extern "C" {
// Caching device allocator: blocks are 2-MiB multiples (256-B multiples below 1 MiB); a
// request reuses the smallest cached block that is at least as large and at most 1/8
// larger, else hipMalloc.  Released blocks are cached up to AM_BLOCK_CACHE bytes per
// context.
static constexpr size_t AM_BLOCK_CACHE = (size_t)64 << 30;

int am_dev_alloc(am_ctx *c, size_t bytes, void **out) {
  if (!c || !out) return AM_ERR_INVALID;
  AM_LOCK(c);
  AM_HIP(hipSetDevice(c->device));
  const size_t want = am_round_up(bytes ? bytes : 16, bytes >= ((size_t)1 << 20) ? ((size_t)2 << 20) : 256);
  auto it = c->free_blocks.lower_bound(want);
  if (it != c->free_blocks.end() && it->first <= want + want / 8) {
    *out = it->second;
    c->free_bytes -= it->first;
    c->free_blocks.erase(it);
    return AM_OK;
  }
  void *p = nullptr;
  hipError_t e = hipMalloc(&p, want);
  if (e != hipSuccess && !c->free_blocks.empty()) {  // out of memory: give the cache back, retry
    (void)hipStreamSynchronize(c->stream);
    for (auto &kv : c->free_blocks) (void)hipFree(kv.second);
    c->free_blocks.clear();
    c->free_bytes = 0;
    e = hipMalloc(&p, want);
  }
  if (e != hipSuccess) {
    am_set_error("hipMalloc(%zu): %s", want, hipGetErrorString(e));
    return AM_ERR_NOMEM;
  }
  c->block_size[p] = want;
  *out = p;
  return AM_OK;
}

void am_dev_release(am_ctx *c, void *p) {
  if (!c || !p) return;
  AM_LOCK(c);
  auto it = c->block_size.find(p);
  if (it == c->block_size.end() || c->free_bytes + it->second > AM_BLOCK_CACHE) {
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    if (it != c->block_size.end()) c->block_size.erase(it);
    (void)hipFree(p);
    return;
  }
  c->free_blocks.emplace(it->second, p);
  c->free_bytes += it->second;
}

int am_dev_free(am_ctx *c, void *p) {
  if (!c) return AM_ERR_INVALID;
  am_dev_release(c, p);
  return AM_OK;
}

int am_memcpy_h2d(am_ctx *c, void *dst, const void *src, size_t bytes) {
  if (!c) return AM_ERR_INVALID;
  AM_LOCK(c);
  if (!bytes) return AM_OK;
  AM_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
  AM_HIP(hipStreamSynchronize(c->stream));
  return AM_OK;
}

int am_memcpy_d2h(am_ctx *c, void *dst, const void *src, size_t bytes) {
  if (!c) return AM_ERR_INVALID;
  AM_LOCK(c);
  if (!bytes) return AM_OK;
  AM_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
  AM_HIP(hipStreamSynchronize(c->stream));
  return AM_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- stores
static int store_alloc(am_store *st, size_t bytes, void **out) {
  void *p = nullptr;
  int rc = am_dev_alloc(st->ctx, bytes, &p);
  if (rc) return rc;
  st->allocs.push_back(p);
  *out = p;
  return AM_OK;
}

template <typename T>
static int upload(am_store *st, const T *src, uint64_t n, uint64_t n_alloc, const T **dst) {
  if (!src) {
    *dst = nullptr;
    return AM_OK;
  }
  void *p = nullptr;
  int rc = store_alloc(st, n_alloc * sizeof(T), &p);
  if (rc) return rc;
  AM_HIP(hipMemsetAsync(p, 0, n_alloc * sizeof(T), st->ctx->stream));
  if (n) AM_HIP(hipMemcpyAsync(p, src, n * sizeof(T), hipMemcpyHostToDevice, st->ctx->stream));
  *dst = (const T *)p;
  return AM_OK;
}

extern "C" {

int am_store_destroy(am_store *st) {
  if (!st) return AM_OK;
  AM_LOCK(st->ctx);
  (void)hipSetDevice(st->ctx->device);
  for (void *p : st->allocs) am_dev_release(st->ctx, p);  // kept for the next store's columns
  delete st;
  return AM_OK;
}

int am_store_create(am_ctx *c, const am_op_log *h, am_store **out) {
  if (!c) return AM_ERR_INVALID;
  AM_LOCK(c);
  if (!c || !h || !out || !h->key_off || !h->key_type || !h->op_meta || !h->commit_time || !h->p0) {
    am_set_error("am_store_create: missing required arrays");
    return AM_ERR_INVALID;
  }
  if (h->n_dc == 0 || h->n_dc > AM_MAX_DC) return AM_ERR_INVALID;
  if (h->n_dc && h->n_ops && !h->snap_vc) return AM_ERR_INVALID;
  AM_HIP(hipSetDevice(c->device));
  am_store *st = new am_store();
  st->ctx = c;
  const uint64_t n_ops = h->n_ops, n_keys = h->n_keys;
  const uint64_t na = am_round_up(n_ops, AM_OP_PAD) + AM_OP_PAD;  // padded so tiles can over-read
  am_op_log &d = st->dev;
  d.n_dc = h->n_dc;
  d.n_keys = n_keys;
  d.n_ops = n_ops;
  d.n_var = h->n_var;
  d.snap_stride = na;
  int rc = AM_OK;
#define UP(field, cnt, cnt_alloc) \
  if (!rc) rc = upload(st, h->field, cnt, cnt_alloc, &d.field)
  UP(key_off, n_keys + 1, n_keys + 1);
  UP(key_id_base, n_keys, n_keys);
  UP(key_type, n_keys, n_keys);
  UP(key_flags, n_keys, n_keys);
  UP(op_meta, n_ops, na);
  UP(commit_time, n_ops, na);
  UP(snap_pres, n_ops, na);
  UP(op_txid, n_ops, na);
  UP(op_id, n_ops, na);
  UP(p0, n_ops, na);
  UP(p1, n_ops, na);
  UP(var_off, h->var_off ? n_ops + 1 : 0, n_ops + 1);
  UP(var_data, h->n_var, h->n_var + 4);
#undef UP
  if (!rc && h->snap_vc) {
    void *p = nullptr;
    rc = store_alloc(st, (size_t)h->n_dc * na * sizeof(uint64_t), &p);
    if (!rc) {
      const uint64_t hs = h->snap_stride ? h->snap_stride : n_ops;
      AM_HIP(hipMemsetAsync(p, 0, (size_t)h->n_dc * na * sizeof(uint64_t), c->stream));
      if (n_ops)
        AM_HIP(hipMemcpy2DAsync(p, na * sizeof(uint64_t), h->snap_vc, hs * sizeof(uint64_t),
                                n_ops * sizeof(uint64_t), h->n_dc, hipMemcpyHostToDevice, c->stream));
      d.snap_vc = (const uint64_t *)p;
    }
  }
  if (!rc) {
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) {
      am_set_error("store upload: %s", hipGetErrorString(e));
      rc = AM_ERR_HIP;
    }
  }
  if (!rc) rc = am_store_pack(st);
  if (rc) {
    am_store_destroy(st);
    return rc;
  }
  *out = st;
  return AM_OK;
}

int am_store_log(const am_store *st, am_op_log *out) {
  if (!st || !out) return AM_ERR_INVALID;
  *out = st->dev;
  return AM_OK;
}

// ---------------------------------------------------------------- hot path
int am_materialize(am_ctx *c, const am_op_log *L, const am_read_batch *B, am_read_result *R) {
  if (!c) return AM_ERR_INVALID;
  AM_LOCK(c);
  AM_HIP(hipSetDevice(c->device));
  return am_launch_materialize(c, L, B, R);
}

uint32_t am_key_partition(int64_t key, uint32_t n_partitions) {
  if (n_partitions == 0) return 0;
  const uint64_t a = key < 0 ? (uint64_t)(-(key + 1)) + 1 : (uint64_t)key;  // abs without UB
  return (uint32_t)(a % n_partitions);
}

// ---------------------------------------------------------------- GST
int am_gst_local_min(am_ctx *c, uint32_t n_dc, uint32_t n_part, const uint64_t *part_vc, const uint32_t *part_pres,
                     const uint8_t *part_undef, uint64_t *lanes) {
  if (!c || !lanes || n_dc == 0 || n_dc > AM_MAX_DC) return AM_ERR_INVALID;
  AM_LOCK(c);
  AM_HIP(hipSetDevice(c->device));
  return am_launch_gst_local_min(c, n_dc, n_part, part_vc, part_pres, part_undef, lanes);
}

int am_gst_finalize(am_ctx *c, uint32_t n_dc, const uint64_t *lanes, uint64_t *last_vc, uint32_t *last_pres, int gr,
                    uint64_t *out_vc, uint32_t *out_pres, uint8_t *changed) {
  if (!c) return AM_ERR_INVALID;
  AM_LOCK(c);
  if (!c || !lanes || !last_vc || !last_pres || !out_vc || !out_pres || n_dc == 0 || n_dc > AM_MAX_DC)
    return AM_ERR_INVALID;
  AM_HIP(hipSetDevice(c->device));
  return am_launch_gst_finalize(c, n_dc, lanes, last_vc, last_pres, gr, out_vc, out_pres, changed);
}

}  // extern "C"
