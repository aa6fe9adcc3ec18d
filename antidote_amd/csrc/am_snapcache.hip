// am_snapcache.hip -- the materializer_vnode snapshot cache on the device, so a batch of
// reads runs the whole of materializer_vnode:internal_read/7 (src/materializer_vnode.erl:
// 371-376) without leaving HBM:
//   k_sc_claim     one read per key and batch (the lowest read index owns the key)
//   k_sc_select    get_from_snapshot_cache/5 (:384-413): no dict yet -> base {ignore,
//                  new()} and is_newest = true; otherwise vector_orddict:get_smaller/2
//                  (src/vector_orddict.erl:75-87): the newest cached snapshot whose
//                  clock is vectorclock:le the read clock; none -> the log cold path
//   am_materialize materialize/4 on the selected bases (every tier of am_plan.hip)
//   k_sc_store     the empty-dict insertion of get_from_snapshot_cache, then
//                  materialize_snapshot/7's write-back (:469-509): only when the key has
//                  ops, LastOpCt /= ignore and WasUpdated, IsNewest and Count >=
//                  MIN_OP_STORE_SS; internal_store_ss/4 (:342-364) with its
//                  NewLastOp - first.last_op_id >= MIN_OP_STORE_SS test;
//                  vector_orddict:insert_bigger/3 (:127-140); snapshot_insert_gc/3's list
//                  pruning (:515-563: at SNAPSHOT_THRESHOLD entries keep SNAPSHOT_MIN)
//   k_sc_release   frees the key claims
// Layout: per key a fixed array of CAP entries, newest first (clock [n_dc] + presence,
// last_op_id, value).  Scalar-valued types (PN counter, LWW register).  The op-cache
// pruning that snapshot_insert_gc also does (prune_ops) is not applied: pruned ops are
// already inside every retained snapshot, so no read's result depends on it (SURVEY.md
// 8(f) rank 1 is the device op-cache GC).
#include "am_wave.h"

using namespace amk;

struct am_snapcache {
  am_ctx *ctx = nullptr;
  uint32_t n_dc = 0;
  uint64_t n_keys = 0;
  uint8_t *cnt = nullptr;      // [n_keys] entries; ABSENT: no snapshot dict yet
  uint32_t *owner = nullptr;   // [n_keys] batch claim (~0: free)
  uint64_t *vc = nullptr;      // [n_keys][CAP][n_dc]
  uint32_t *pres = nullptr;    // [n_keys][CAP]
  int64_t *last_op = nullptr;  // [n_keys][CAP]
  int64_t *v0 = nullptr;       // [n_keys][CAP]
  uint64_t *v1 = nullptr;      // [n_keys][CAP]
  uint8_t *vflag = nullptr;    // [n_keys][CAP]
  std::vector<void *> allocs;
};

namespace {

constexpr uint32_t CAP = AM_SNAPSHOT_THRESHOLD;   // insert_bigger + gc keep at most THRESHOLD - 1
constexpr uint32_t SMIN = AM_SNAPSHOT_MIN;
constexpr uint32_t MIN_OP_STORE_SS = AM_MIN_OP_STORE_SS;
constexpr uint8_t ABSENT = 0xFF;
// per-read selection codes (scratch)
enum : uint8_t { SEL_CACHED = 0, SEL_NEW_DICT = 1, SEL_COLD = 2, SEL_DUP = 3, SEL_BAD = 4 };

struct ScView {  // kernel-side copy of the cache pointers
  uint32_t n_dc;
  uint64_t n_keys;
  uint8_t *cnt;
  uint32_t *owner;
  uint64_t *vc;
  uint32_t *pres;
  int64_t *last_op, *v0;
  uint64_t *v1;
  uint8_t *vflag;
};
// selected bases (scratch, columns of the batch handed to am_materialize)
struct ScSel {
  uint8_t *code, *newest, *base_ignore, *vflag;
  uint64_t *base_vc, *v1;
  uint32_t *base_pres;
  int64_t *base_last_op, *v0;
};

__device__ __forceinline__ uint64_t clk(const uint64_t *vc, uint32_t pres, uint32_t d) {
  return ((pres >> d) & 1u) ? vc[d] : 0;
}

__global__ void k_sc_claim(ScView C, am_read_batch B) {
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < B.n_reads; r += (uint64_t)gridDim.x * blockDim.x)
    if (B.key[r] < C.n_keys) atomicMin(&C.owner[B.key[r]], (uint32_t)r);
}

__global__ void k_sc_release(ScView C, am_read_batch B) {
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < B.n_reads; r += (uint64_t)gridDim.x * blockDim.x)
    if (B.key[r] < C.n_keys) C.owner[B.key[r]] = 0xFFFFFFFFu;
}

__global__ void k_sc_select(ScView C, am_read_batch B, ScSel S) {
  const uint32_t nd = C.n_dc;
  const uint32_t all = nd >= 32 ? 0xFFFFFFFFu : ((1u << nd) - 1u);
  const uint64_t n = B.n_reads;
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t key = B.key[r];
    const uint32_t t = B.type[r];
    uint8_t code = SEL_NEW_DICT, newest = 1;
    uint32_t bpres = 0;
    int64_t blast = 0, bv0 = 0;
    uint64_t bv1 = 0;
    uint8_t bvf = t == AM_LWW ? 1 : 0, bign = 1;  // new(): 0 / {0, <<>>}
    uint32_t sel = CAP;
    if (key >= C.n_keys || (t != AM_PN && t != AM_LWW)) {
      code = SEL_BAD;
    } else if (C.owner[key] != (uint32_t)r) {
      code = SEL_DUP;
    } else if (C.cnt[key] != ABSENT) {
      const uint64_t ridx = B.per_read_clock ? r : 0, rstride = B.per_read_clock ? n : 1;
      const uint32_t spres = B.read_pres[ridx] & all;
      const uint32_t ne = C.cnt[key];
      for (uint32_t e = 0; e < ne && sel == CAP; ++e) {  // vector_orddict:get_smaller: newest first
        const uint64_t slot = key * CAP + e;
        const uint32_t ep = C.pres[slot] & all;
        bool le = true;  // vectorclock:le(Entry, ReadClock): every DC of either, missing = 0
        for (uint32_t d = 0; d < nd && le; ++d) {
          const uint64_t x = clk(C.vc + slot * nd, ep, d);
          const uint64_t y = ((spres >> d) & 1u) ? B.read_vc[(uint64_t)d * rstride + ridx] : 0;
          le = x <= y;
        }
        if (le) sel = e;
      }
      if (sel == CAP) {
        code = SEL_COLD;  // get_from_snapshot_log: the log path, not the cache
      } else {
        const uint64_t slot = key * CAP + sel;
        code = SEL_CACHED;
        newest = sel == 0;
        bign = 0;
        bpres = C.pres[slot] & all;
        for (uint32_t d = 0; d < nd; ++d) S.base_vc[(uint64_t)d * n + r] = clk(C.vc + slot * nd, bpres, d);
        blast = C.last_op[slot];
        bv0 = C.v0[slot];
        bv1 = C.v1[slot];
        bvf = C.vflag[slot];
      }
    }
    if (bign)
      for (uint32_t d = 0; d < nd; ++d) S.base_vc[(uint64_t)d * n + r] = 0;
    S.code[r] = code;
    S.newest[r] = newest;
    S.base_ignore[r] = bign;
    S.base_pres[r] = bpres;
    S.base_last_op[r] = blast;
    S.v0[r] = bv0;
    S.v1[r] = bv1;
    S.vflag[r] = bvf;
  }
}

__global__ void k_sc_store(ScView C, am_op_log L, am_read_batch B, am_read_result R, ScSel S) {
  const uint32_t nd = C.n_dc;
  const uint64_t n = B.n_reads;
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (uint64_t)gridDim.x * blockDim.x) {
    const uint8_t code = S.code[r];
    if (code == SEL_BAD) {
      if (R.status[r] == AM_OK) R.status[r] = AM_ERR_UNSUPPORTED;  // set / bcounter values: not cached here
      continue;
    }
    if (code == SEL_DUP) {
      R.status[r] = AM_ERR_INVALID;
      continue;
    }
    if (code == SEL_COLD) {
      R.status[r] = AM_ERR_COLD_PATH;
      continue;
    }
    const uint64_t key = B.key[r];
    const uint32_t t = B.type[r];
    uint32_t ne = C.cnt[key];
    if (code == SEL_NEW_DICT) {  // store_snapshot(TxId, Key, Empty, vectorclock:new(), false)
      const uint64_t s0 = key * CAP;
      C.pres[s0] = 0;
      for (uint32_t d = 0; d < nd; ++d) C.vc[s0 * nd + d] = 0;
      C.last_op[s0] = 0;
      C.v0[s0] = 0;
      C.v1[s0] = 0;
      C.vflag[s0] = t == AM_LWW ? 1 : 0;
      ne = 1;
      C.cnt[key] = 1;
    }
    // materialize_snapshot/7: number_of_ops == 0 returns the base; errors and
    // CommitTime == ignore return without caching
    if (R.status[r] != AM_OK || L.key_off[key + 1] == L.key_off[key] || R.last_ct_ignore[r]) continue;
    if (!(R.is_new_ss[r] && S.newest[r] && R.count[r] >= MIN_OP_STORE_SS)) continue;
    // internal_store_ss/4: ShouldInsert = NewLastOp - first.last_op_id >= MIN_OP_STORE_SS
    const uint64_t s0 = key * CAP;
    const int64_t nlo = R.new_last_op[r];
    if (!(nlo - C.last_op[s0] >= (int64_t)MIN_OP_STORE_SS)) continue;
    // vector_orddict:insert_bigger: prepend iff not vectorclock:le(New, First)
    const uint32_t np = R.last_ct_pres[r];
    const uint32_t fp = C.pres[s0];
    bool le = true;
    for (uint32_t d = 0; d < nd && le; ++d) {
      const uint64_t x = ((np >> d) & 1u) ? R.last_ct[(uint64_t)d * n + r] : 0;
      le = x <= clk(C.vc + s0 * nd, fp, d);
    }
    if (le) continue;
    // snapshot_insert_gc: at SNAPSHOT_THRESHOLD entries keep the newest SNAPSHOT_MIN
    const uint32_t grown = ne + 1;
    const uint32_t keep = grown >= CAP ? SMIN : grown;
    for (uint32_t e = keep - 1; e >= 1; --e) {  // shift right by one (newest first)
      const uint64_t dst = s0 + e, src = s0 + e - 1;
      for (uint32_t d = 0; d < nd; ++d) C.vc[dst * nd + d] = C.vc[src * nd + d];
      C.pres[dst] = C.pres[src];
      C.last_op[dst] = C.last_op[src];
      C.v0[dst] = C.v0[src];
      C.v1[dst] = C.v1[src];
      C.vflag[dst] = C.vflag[src];
    }
    for (uint32_t d = 0; d < nd; ++d) C.vc[s0 * nd + d] = ((np >> d) & 1u) ? R.last_ct[(uint64_t)d * n + r] : 0;
    C.pres[s0] = np;
    C.last_op[s0] = nlo;
    C.v0[s0] = R.value.v0[r];
    C.v1[s0] = t == AM_LWW ? R.value.v1[r] : 0;
    C.vflag[s0] = t == AM_LWW ? R.value.vflag[r] : 0;
    C.cnt[key] = (uint8_t)keep;
  }
}

ScView view(const am_snapcache *c) {
  return ScView{c->n_dc, c->n_keys, c->cnt, c->owner, c->vc, c->pres, c->last_op, c->v0, c->v1, c->vflag};
}
unsigned grid(uint64_t n) { return (unsigned)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096); }

// snapshot_insert_gc/4's threshold (src/materializer_vnode.erl:522-527): PrunedSnapshots =
// sublist(Dict, 1, SNAPSHOT_MIN) (newest first), CommitTime = vectorclock:min over them
// (dict merge: a DC present in any of the clocks is kept, with the min over those having it)
__global__ void k_sc_threshold(ScView C, uint8_t *mask, uint64_t *thr_vc, uint32_t *thr_pres) {
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < C.n_keys;
       k += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t cnt = C.cnt[k];
    const uint32_t m = (cnt == ABSENT) ? 0 : (cnt < SMIN ? cnt : SMIN);
    uint32_t pres = 0;
    for (uint32_t e = 0; e < m; ++e) pres |= C.pres[k * CAP + e];
    for (uint32_t d = 0; d < C.n_dc; ++d) {
      uint64_t t = ~0ull;
      for (uint32_t e = 0; e < m; ++e)
        if ((C.pres[k * CAP + e] >> d) & 1u) {
          const uint64_t v = C.vc[(k * CAP + e) * C.n_dc + d];
          t = v < t ? v : t;
        }
      thr_vc[(uint64_t)d * C.n_keys + k] = ((pres >> d) & 1u) ? t : 0;
    }
    thr_pres[k] = pres;
    mask[k] = m ? 1 : 0;
  }
}

}  // namespace

extern "C" {

int am_snapcache_create(am_ctx *ctx, uint32_t n_dc, uint64_t n_keys, am_snapcache **out) {
  if (!ctx || !out || n_dc == 0 || n_dc > AM_MAX_DC) return AM_ERR_INVALID;
  am_snapcache *c = new am_snapcache();
  c->ctx = ctx;
  c->n_dc = n_dc;
  c->n_keys = n_keys;
  const uint64_t ne = n_keys * CAP + 1;
  auto alloc = [&](size_t bytes, void **p) {
    int rc = am_dev_alloc(ctx, bytes, p);
    if (!rc) c->allocs.push_back(*p);
    return rc;
  };
  int rc = alloc(n_keys + 16, (void **)&c->cnt);
  if (!rc) rc = alloc((n_keys + 1) * 4, (void **)&c->owner);
  if (!rc) rc = alloc(ne * n_dc * 8, (void **)&c->vc);
  if (!rc) rc = alloc(ne * 4, (void **)&c->pres);
  if (!rc) rc = alloc(ne * 8, (void **)&c->last_op);
  if (!rc) rc = alloc(ne * 8, (void **)&c->v0);
  if (!rc) rc = alloc(ne * 8, (void **)&c->v1);
  if (!rc) rc = alloc(ne, (void **)&c->vflag);
  if (!rc && hipMemsetAsync(c->cnt, ABSENT, n_keys + 16, ctx->stream) != hipSuccess) rc = AM_ERR_HIP;
  if (!rc && hipMemsetAsync(c->owner, 0xFF, (n_keys + 1) * 4, ctx->stream) != hipSuccess) rc = AM_ERR_HIP;
  if (rc) {
    am_snapcache_destroy(c);
    return rc;
  }
  *out = c;
  return AM_OK;
}

int am_snapcache_destroy(am_snapcache *c) {
  if (!c) return AM_OK;
  if (c->ctx) (void)hipStreamSynchronize(c->ctx->stream);
  for (void *p : c->allocs) (void)hipFree(p);
  delete c;
  return AM_OK;
}

int am_snapcache_read(am_ctx *ctx, am_snapcache *c, const am_op_log *L, const am_read_batch *B, am_read_result *R) {
  if (!ctx || !c || !L || !B || !R || c->ctx != ctx) return AM_ERR_INVALID;
  if (L->n_dc != c->n_dc || L->n_keys > c->n_keys) {
    am_set_error("snapshot cache: n_dc / n_keys do not match the log");
    return AM_ERR_INVALID;
  }
  if (!R->value.v0 || !R->value.v1 || !R->value.vflag) {
    am_set_error("snapshot cache reads need value.v0/v1/vflag");
    return AM_ERR_INVALID;
  }
  const uint64_t n = B->n_reads;
  if (n == 0) return AM_OK;
  const uint32_t nd = c->n_dc;
  // scratch: code, newest, base_ignore, vflag [n] u8 | base_pres [n] u32 | base_last_op, v0, v1 [n] u64 | base_vc [nd][n]
  const size_t bytes = n * (4 + 4 + 3 * 8 + (size_t)nd * 8) + 1024;
  void *scr = nullptr;
  int rc = am_ctx_scratch(ctx, AM_SCR_SNAP, bytes, &scr);
  if (rc) return rc;
  char *p = (char *)scr;
  auto take = [&](size_t b) {
    char *q = p;
    p += (b + 255) & ~(size_t)255;
    return q;
  };
  ScSel S;
  S.base_last_op = (int64_t *)take(n * 8);
  S.v0 = (int64_t *)take(n * 8);
  S.v1 = (uint64_t *)take(n * 8);
  S.base_vc = (uint64_t *)take(n * nd * 8);
  S.base_pres = (uint32_t *)take(n * 4);
  S.code = (uint8_t *)take(n);
  S.newest = (uint8_t *)take(n);
  S.base_ignore = (uint8_t *)take(n);
  S.vflag = (uint8_t *)take(n);
  const ScView V = view(c);
  hipLaunchKernelGGL(k_sc_claim, dim3(grid(n)), dim3(256), 0, ctx->stream, V, *B);
  hipLaunchKernelGGL(k_sc_select, dim3(grid(n)), dim3(256), 0, ctx->stream, V, *B, S);
  AM_HIP(hipGetLastError());
  am_read_batch db = *B;
  db.base_ignore = S.base_ignore;
  db.base_vc = S.base_vc;
  db.base_pres = S.base_pres;
  db.base_last_op = S.base_last_op;
  db.base.v0 = S.v0;
  db.base.v1 = S.v1;
  db.base.vflag = S.vflag;
  rc = am_launch_materialize(ctx, L, &db, R);
  if (rc == AM_OK) {
    hipLaunchKernelGGL(k_sc_store, dim3(grid(n)), dim3(256), 0, ctx->stream, V, *L, *B, *R, S);
    AM_HIP(hipGetLastError());
  }
  hipLaunchKernelGGL(k_sc_release, dim3(grid(n)), dim3(256), 0, ctx->stream, V, *B);
  AM_HIP(hipGetLastError());
  return rc;
}

int am_snapcache_gc_threshold(am_ctx *ctx, const am_snapcache *c, uint8_t *mask, uint64_t *thr_vc,
                              uint32_t *thr_pres) {
  if (!ctx || !c || !mask || !thr_vc || !thr_pres) return AM_ERR_INVALID;
  AM_HIP(hipSetDevice(ctx->device));
  if (c->n_keys == 0) return AM_OK;
  hipLaunchKernelGGL(k_sc_threshold, dim3(grid(c->n_keys)), dim3(256), 0, ctx->stream, view(c), mask, thr_vc, thr_pres);
  AM_HIP(hipGetLastError());
  return AM_OK;
}

int am_snapcache_get(am_ctx *ctx, const am_snapcache *c, uint64_t key, uint32_t *n_entries, uint64_t *vc,
                     uint32_t *pres, int64_t *last_op, int64_t *v0, uint64_t *v1, uint8_t *vflag) {
  if (!ctx || !c || !n_entries || key >= c->n_keys) return AM_ERR_INVALID;
  uint8_t cnt = 0;
  const uint64_t s0 = key * CAP, nd = c->n_dc;
  AM_HIP(hipMemcpyAsync(&cnt, c->cnt + key, 1, hipMemcpyDeviceToHost, ctx->stream));
  if (vc) AM_HIP(hipMemcpyAsync(vc, c->vc + s0 * nd, CAP * nd * 8, hipMemcpyDeviceToHost, ctx->stream));
  if (pres) AM_HIP(hipMemcpyAsync(pres, c->pres + s0, CAP * 4, hipMemcpyDeviceToHost, ctx->stream));
  if (last_op) AM_HIP(hipMemcpyAsync(last_op, c->last_op + s0, CAP * 8, hipMemcpyDeviceToHost, ctx->stream));
  if (v0) AM_HIP(hipMemcpyAsync(v0, c->v0 + s0, CAP * 8, hipMemcpyDeviceToHost, ctx->stream));
  if (v1) AM_HIP(hipMemcpyAsync(v1, c->v1 + s0, CAP * 8, hipMemcpyDeviceToHost, ctx->stream));
  if (vflag) AM_HIP(hipMemcpyAsync(vflag, c->vflag + s0, CAP, hipMemcpyDeviceToHost, ctx->stream));
  AM_HIP(hipStreamSynchronize(ctx->stream));
  *n_entries = cnt == ABSENT ? AM_SNAPCACHE_ABSENT : cnt;
  return AM_OK;
}

}  // extern "C"
