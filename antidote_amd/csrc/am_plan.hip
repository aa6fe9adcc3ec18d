// am_plan.hip -- the batch planner behind am_materialize.
//
// A read batch from a partition's read servers mixes CRDT types (each
// materializer_vnode:read/6 call names its Type, src/materializer_vnode.erl:97-102).
// Every type has its own kernels (k_stream + row tier: PN counter, LWW register;
// am_group.hip: add-wins set, MV register; row tier + k_sets: bounded counter; k_sets /
// am_big.hip: set reads the group tier does not take), so a mixed batch is split on the
// device, never on the host:
//   k_plan_count    per 1024-read block: class histogram (class = kernel the read needs;
//                   reads with an unknown type or key get their status here); the block
//                   claims its slice of every class with one atomicAdd per class
//   k_plan_scatter  partition of the read indices by class (wave ballots; blocks keep their
//                   reads in order, the order of the blocks inside a class is the claim
//                   order -- every read writes only its own outputs, so results do not
//                   depend on it) and the [begin, end) range of every class
// and each type kernel then runs over its class range (am_sel).  The ranges stay in
// device memory: kernels are launched with a resident-capacity grid and read their
// count at start, so the planner adds no host round trip.
//
// Single-type batches (type_hint != 0) skip the planner.  Set types may need the
// big-read path, which sizes its scratch on the host (one synchronization).  In a mixed
// batch every set type's chain runs on a stream of its own (am_ctx::sub), joined back
// before the call returns: a type's latency-bound tiers overlap the other types' tiers.
#include "am_wave.h"

using namespace amk;

namespace {

constexpr int PB = 256;              // planner block
constexpr int PER = 4;               // reads per thread
constexpr uint32_t PCHUNK = PB * PER;
// classes: 1..5 = the type, 6 = done (status written), 0 = an MV read of a key in the chunked
// big view when `mvbig` (the big-read tier takes it straight from the batch, beside the other
// tiers; class 0 starts at 0, so its list is the plan's index array and its count range[1])
constexpr int NCLS = 8;
constexpr uint32_t CLS_MVBIG = 0, CLS_DONE = 6;

__device__ __forceinline__ uint32_t read_class(const am_op_log &L, const am_read_batch &B, am_read_result &R,
                                               uint64_t r, bool write_status, bool mvbig) {
  const uint32_t t = B.type[r];
  const uint64_t key = B.key[r];
  if (t < AM_PN || t > AM_BCOUNTER || key >= L.n_keys) {
    if (write_status) R.status[r] = AM_ERR_INVALID;
    return CLS_DONE;
  }
  if (mvbig && t == AM_MVREG && L.key_type[key] == AM_MVREG && am_ngrp_big(L.key_ngrp[key])) return CLS_MVBIG;
  return t;
}

// the planner's input: the whole batch, or a selection (the lane tier's hand-off list)
__device__ __forceinline__ uint64_t in_count(const am_read_batch &B, am_sel in) {
  return in.idx ? (uint64_t)(uniform_u32(in.range[1]) - uniform_u32(in.range[0])) : B.n_reads;
}
__device__ __forceinline__ uint64_t in_read(am_sel in, uint64_t i) {
  return in.idx ? (uint64_t)in.idx[in.range[0] + i] : i;
}

__global__ void __launch_bounds__(PB) k_plan_count(am_op_log L, am_read_batch B, am_read_result R, am_sel in,
                                                   uint32_t *cnt, uint32_t *tot, bool write_status, bool mvbig) {
  __shared__ uint32_t c[NCLS];
  if (threadIdx.x < NCLS) c[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * PCHUNK, nin = in_count(B, in);
  for (int j = 0; j < PER; ++j) {
    const uint64_t i = base + (uint64_t)j * PB + threadIdx.x;
    if (i < nin) atomicAdd(&c[read_class(L, B, R, in_read(in, i), write_status, mvbig)], 1u);
  }
  __syncthreads();
  if (threadIdx.x < NCLS) cnt[(uint64_t)blockIdx.x * NCLS + threadIdx.x] = atomicAdd(&tot[threadIdx.x], c[threadIdx.x]);
}

__global__ void __launch_bounds__(PB) k_plan_scatter(am_op_log L, am_read_batch B, am_read_result R, am_sel in,
                                                     const uint32_t *off, const uint32_t *tot, uint32_t *range,
                                                     uint32_t *idx, bool mvbig) {
  __shared__ uint32_t run[NCLS];
  __shared__ uint32_t wcnt[PB / WAVE][NCLS];
  const uint32_t tid = threadIdx.x, w = tid / WAVE, lane = tid % WAVE;
  if (tid < NCLS) {  // class start = the totals of the classes before it
    uint32_t start = 0;
    for (uint32_t k = 0; k < tid; ++k) start += tot[k];
    run[tid] = start + off[(uint64_t)blockIdx.x * NCLS + tid];
    if (blockIdx.x == 0) range[2 * tid] = start, range[2 * tid + 1] = start + tot[tid];
  }
  const uint64_t base = (uint64_t)blockIdx.x * PCHUNK, nin = in_count(B, in);
  for (int j = 0; j < PER; ++j) {
    const uint64_t i = base + (uint64_t)j * PB + tid;
    const uint64_t r = i < nin ? in_read(in, i) : 0;
    const uint32_t c = i < nin ? read_class(L, B, R, r, false, mvbig) : NCLS;
    uint32_t rank = 0;
    for (uint32_t k = 0; k < NCLS; ++k) {
      const uint64_t m = __ballot(c == k);
      if (c == k) rank = __popcll(m & ((1ull << lane) - 1));
      if (lane == 0) wcnt[w][k] = __popcll(m);
    }
    __syncthreads();
    if (c < NCLS) {
      uint32_t before = run[c];
      for (uint32_t v = 0; v < w; ++v) before += wcnt[v][c];
      idx[before + rank] = (uint32_t)r;
    }
    __syncthreads();
    if (tid < NCLS) {
      uint32_t t = 0;
      for (int v = 0; v < PB / WAVE; ++v) t += wcnt[v][tid];
      run[tid] += t;
    }
    __syncthreads();
  }
}

// bit t: a key of type t; TYPES_MVBIG: an MV key in the chunked big view
constexpr uint32_t TYPES_MVBIG = 1u << 31;
__global__ void __launch_bounds__(PB) k_type_mask(const uint8_t *key_type, const uint32_t *key_ngrp, uint64_t n,
                                                  uint32_t *out) {
  uint32_t m = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * PB + threadIdx.x; i < n; i += (uint64_t)gridDim.x * PB) {
    const uint32_t t = key_type[i];
    m |= t < 31 ? 1u << t : 0u;
    if (t == AM_MVREG && key_ngrp && am_ngrp_big(key_ngrp[i])) m |= TYPES_MVBIG;
  }
  m = wave_or_u32(m);
  if ((threadIdx.x & (WAVE - 1)) == 0 && m) atomicOr(out, m);
}

// The types present in the log's keys (one pass + readback per key_type array, cached on the
// context).  It only picks the order of the mixed batch's chains and whether the big MV reads
// are planned early: a stale entry (a store rebuilt over a reused block) costs time, never a
// result.
int log_types(am_ctx *ctx, const am_op_log *L, uint32_t *mask) {
  auto it = ctx->type_masks.find(L->key_type);
  if (it != ctx->type_masks.end() && it->second.first == L->n_keys) {
    *mask = it->second.second;
    return AM_OK;
  }
  void *w = nullptr;
  if (int rc = am_ctx_scratch(ctx, AM_SCR_MISC, 256, &w)) return rc;
  AM_HIP(hipMemsetAsync(w, 0, sizeof(uint64_t), ctx->stream));
  const uint64_t cap = (uint64_t)ctx->n_cu * 4, nb = (L->n_keys + PB - 1) / PB;
  if (nb)
    hipLaunchKernelGGL(k_type_mask, dim3((unsigned)(nb < cap ? nb : cap)), dim3(PB), 0, ctx->stream, L->key_type,
                       L->key_ngrp, L->n_keys, (uint32_t *)w);
  AM_HIP(hipGetLastError());
  uint64_t h = 0;
  if (int rc = am_ctx_fetch(ctx, w, 1, &h)) return rc;
  if (ctx->type_masks.size() >= 64) ctx->type_masks.clear();
  ctx->type_masks[L->key_type] = {L->n_keys, (uint32_t)h};
  *mask = (uint32_t)h;
  return AM_OK;
}

// Short-read limit of the row tier (am_rows.hip): at most 64 ops (one 16-lane row, 4 steps)
// for PN / LWW; 48 for the bounded counter (longer reads: the wave tier, am_bcwave.hip --
// on C5 48 measured 1.5 % faster than 127 and 36 % faster than sending every read to the
// wave tier).  The row's 64-bit LDS slot sums stay exact up to 127 amounts below 2^56.
constexpr uint32_t ROWS_SCALAR = 64, ROWS_BC = 48;

// PN / LWW over selection S: k_stream takes the long reads and marks the short ones in a
// per-batch mask (rows_buf + 64) for the row tier, which skips batches without any.
int run_scalar(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S, uint32_t type,
               uint32_t *rows_buf) {
  am_rows_cfg H;
  H.short_max = ROWS_SCALAR;
  H.mask = (uint64_t *)(rows_buf + 64);
  int rc = am_launch_stream_skip(ctx, L, B, R, S, type, H);
  if (rc) return rc;
  return am_launch_rows(ctx, L, B, R, S, type, H);
}

// Set types over selection S.
//   add-wins set / MV register: token-group tier, row kernel (short logs) -> wave kernel ->
//     workgroup kernel -> (hand-off lists) LDS-sort tier k_sets -> (retry list) big-read tier
//   bounded counter: row tier -> (hand-off lists) wave tier (am_bcwave.hip) -> k_sets ->
//     (retry list) big-read tier
// rows_buf / grp_buf (two lists): [0] = 0, [1] = hand-off count, list at +64.
// run_sets_front: every tier up to k_sets, the big-read tier's retry list in *retry_out.
int run_sets_front(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S,
                   uint32_t type, uint32_t *retry_buf, uint32_t *rows_buf, uint32_t *grp_buf, bool lanes_done,
                   am_retry *retry_out) {
  am_retry retry;
  retry.count = retry_buf;
  retry.list = retry_buf + 1;
  AM_HIP(hipMemsetAsync(retry.count, 0, sizeof(uint32_t), ctx->stream));
  int rc;
  am_sel cur = S;
  if (type == AM_BCOUNTER) {
    AM_HIP(hipMemsetAsync(rows_buf, 0, 2 * sizeof(uint32_t), ctx->stream));
    if (am_bcrows_applies(L, B, R)) {  // short reads: the touched slots only (am_bcrows.hip)
      am_retry nx;
      nx.count = rows_buf + 1;
      nx.list = rows_buf + 64;
      rc = am_launch_bcrows(ctx, L, B, R, S, nx);
    } else {
      am_rows_cfg C;
      C.short_max = ROWS_BC;
      C.list = rows_buf + 64;
      C.count = rows_buf + 1;
      rc = am_launch_rows(ctx, L, B, R, S, type, C);
    }
    if (rc) return rc;
    cur.idx = rows_buf + 64;
    cur.range = rows_buf;
    if (grp_buf && am_bcwave_applies(L, R)) {  // wave per read up to its limit (am_bcwave.hip)
      AM_HIP(hipMemsetAsync(grp_buf, 0, 2 * sizeof(uint32_t), ctx->stream));
      am_retry nx;
      nx.count = grp_buf + 1;
      nx.list = grp_buf + 64;
      rc = am_launch_bcwave(ctx, L, B, R, cur, nx);
      if (rc) return rc;
      // the wave tier hands on only logs above AM_BCWAVE_OPS, which the LDS-sort tier would pass
      // to the big-read tier whole: its list is the big tier's retry list (C5: k_sets over that
      // list held the bounded-counter chain ~0.25 ms)
      static_assert(AM_SETS_BIG_OPS <= AM_BCWAVE_OPS, "k_sets would take some of the wave tier's hand-offs");
      *retry_out = nx;
      return AM_OK;
    }
  } else if (grp_buf && am_group_applies(L, R, type)) {
    // wave -> lane (or, off the packed view, row) -> workgroup kernels; each hands what it
    // does not take to the next.  The wave kernel goes first and hands the short reads on,
    // so a batch of long logs (C3) is not passed over by the lane kernel, whose hand-off
    // atomics then serialize (one per wave on one counter).  Over a mixed batch the lane
    // tier already ran.
    uint32_t *bufs[3] = {rows_buf, grp_buf, grp_buf + (B->n_reads + 64)};
    for (int k = 0; k < 3; ++k) AM_HIP(hipMemsetAsync(bufs[k], 0, 2 * sizeof(uint32_t), ctx->stream));
    const uint32_t lanes = lanes_done ? 0u : am_lane_accept(L, R, 1u << type);
    const int tiers[3] = {AM_GRP_WAVE | (lanes ? AM_GRP_HAND_SHORT : 0), AM_GRP_ROW, AM_GRP_WG};
    for (int k = 0; k < 3; ++k) {
      if (k == 1 && lanes_done) continue;  // the short reads were the lane tier's already
      am_retry nx;
      nx.count = bufs[k] + 1;
      nx.list = bufs[k] + 64;
      rc = (k == 1 && lanes) ? am_launch_lanes(ctx, L, B, R, cur, nx, lanes)
                             : am_launch_group(ctx, L, B, R, cur, type, nx, tiers[k]);
      if (rc) return rc;
      cur.idx = nx.list;
      cur.range = bufs[k];
    }
  }
  *retry_out = retry;
  return am_launch_sets(ctx, L, B, R, cur, type, retry);
}

int run_sets(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S, uint32_t type,
             uint32_t *retry_buf, uint32_t *rows_buf, uint32_t *grp_buf, bool lanes_done) {
  am_retry retry;
  const int rc = run_sets_front(ctx, L, B, R, S, type, retry_buf, rows_buf, grp_buf, lanes_done, &retry);
  return rc ? rc : am_launch_big(ctx, L, B, R, type, retry);
}

// The set chains' big tiers, each launched once its chain's front has drained (its hand-off
// count is read back to size the big tier): in the order the chains finish, not in type order
// -- a host readback that waits on a slow chain would hold back a finished one's big tier
// (C5: the bounded-counter chain drains ~1 ms before the MV chain).  Between polls the host
// blocks on one chain's event instead of spinning.
int launch_bigs_when_ready(am_ctx *const sub[3], const am_op_log *L, const am_read_batch *B, am_read_result *R,
                           const am_retry retry[3]) {
  bool pend[3];
  for (int i = 0; i < 3; ++i) {
    pend[i] = sub[i] != nullptr;
    if (pend[i]) AM_HIP(hipEventRecord(sub[i]->ev1, sub[i]->stream));
  }
  for (int left = pend[0] + pend[1] + pend[2]; left;) {
    int done = 0;
    for (int i = 0; i < 3; ++i) {
      if (!pend[i]) continue;
      const hipError_t q = hipEventQuery(sub[i]->ev1);
      if (q == hipErrorNotReady) continue;
      AM_HIP(q);
      pend[i] = false, --left, ++done;
      if (int rc = am_launch_big(sub[i], L, B, R, AM_AWSET + (uint32_t)i, retry[i])) return rc;
    }
    if (left && !done) {  // block on the chain expected to drain first (bounded counter, then AW, MV)
      // rather than spin a host core beside the RCCL / read-server threads
      for (int i : {2, 0, 1})
        if (pend[i]) {
          AM_HIP(hipEventSynchronize(sub[i]->ev1));
          break;
        }
    }
  }
  return AM_OK;
}

}  // namespace

int am_launch_materialize(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R) {
  if (!ctx || !L || !B || !R) return AM_ERR_INVALID;
  if (L->n_dc == 0 || L->n_dc > AM_MAX_DC) {
    am_set_error("n_dc=%u out of range", L->n_dc);
    return AM_ERR_INVALID;
  }
  const uint64_t stride = L->snap_stride ? L->snap_stride : L->n_ops;
  if ((stride & 3) || (reinterpret_cast<uintptr_t>(L->commit_time) & 15) ||
      (reinterpret_cast<uintptr_t>(L->snap_vc) & 15) || (reinterpret_cast<uintptr_t>(L->p0) & 15) ||
      (reinterpret_cast<uintptr_t>(L->op_meta) & 3)) {
    am_set_error("device log must be 16-byte aligned with snap_stride %% 4 == 0 (use am_store_create)");
    return AM_ERR_INVALID;
  }
  const uint64_t n = B->n_reads;
  if (n == 0) return AM_OK;
  if (n > 0xFFFFFFF0ull) {
    am_set_error("n_reads %llu exceeds the 32-bit read index of one batch", (unsigned long long)n);
    return AM_ERR_INVALID;
  }
  const am_sel all{};
  void *rows_scr = nullptr, *grp_scr = nullptr;
  {
    int rc = am_ctx_scratch(ctx, AM_SCR_ROWS, (n + 64) * sizeof(uint32_t), &rows_scr);
    if (!rc && B->type_hint >= AM_AWSET)
      rc = am_ctx_scratch(ctx, AM_SCR_GRP, 2 * (n + 64) * sizeof(uint32_t), &grp_scr);
    if (rc) return rc;
  }
  if (B->type_hint == AM_PN || B->type_hint == AM_LWW)
    return run_scalar(ctx, L, B, R, all, B->type_hint, (uint32_t *)rows_scr);
  if (B->type_hint == AM_AWSET || B->type_hint == AM_MVREG || B->type_hint == AM_BCOUNTER) {
    void *scr = nullptr;
    int rc = am_ctx_scratch(ctx, AM_SCR_PLAN, (n + 64) * sizeof(uint32_t), &scr);
    if (rc) return rc;
    return run_sets(ctx, L, B, R, all, B->type_hint, (uint32_t *)scr, (uint32_t *)rows_scr, (uint32_t *)grp_scr,
                    false);
  }
  if (B->type_hint != 0) {
    am_set_error("type_hint %u not supported", B->type_hint);
    return AM_ERR_UNSUPPORTED;
  }

  // ---- mixed batch: the lane tier takes the short reads of every type it can in one
  //      launch; the planner partitions the rest by class on the device.  The set types'
  //      chains run on the sub-contexts' streams (one per type, own scratch), the scalar
  //      types' on this one: the chains share only the planner's selection, so one type's
  //      tiers fill the machine while another's drain.  Bounded-counter reads never go to
  //      the lane tier, so their chain is planned from the whole batch on its own stream
  //      and starts beside the lane tier when the log holds bounded-counter keys (on C5
  //      -4.5 %; run over a log without them it cost C4 13 %). ----
  const uint32_t lanes = am_lane_accept(L, R, (1u << AM_PN) | (1u << AM_LWW) | (1u << AM_AWSET) | (1u << AM_MVREG));
  am_ctx *sub[3] = {};
  am_retry retry[3];
  am_ctx *ms = nullptr;  // the early big-MV tier's sub-context
  int rc = AM_OK;
  auto join = [&]() {
    for (am_ctx *s : sub)
      if (s && hipEventRecord(s->ev0, s->stream) == hipSuccess) (void)hipStreamWaitEvent(ctx->stream, s->ev0, 0);
    if (ms && hipEventRecord(ms->ev0, ms->stream) == hipSuccess) (void)hipStreamWaitEvent(ctx->stream, ms->ev0, 0);
  };
  // type t's set chain over class range `range` of selection idx, on its sub-context
  auto start_chain = [&](uint32_t t, const uint32_t *idx, const uint32_t *range, bool forked) -> int {
    am_ctx *s = am_ctx_sub(ctx, (int)(t - AM_AWSET));
    if (!s) return AM_ERR_HIP;
    if (!forked) AM_HIP(hipStreamWaitEvent(s->stream, ctx->ev_fork, 0));
    sub[t - AM_AWSET] = s;
    s->grp_hint_in = ctx->grp_hint_in;
    s->tee_a = ctx->tee_a, s->tee_b = ctx->tee_b, s->tee_g = ctx->tee_g, s->tee_shift = ctx->tee_shift;
    s->tee_done = ctx->tee_done;
    void *sr = nullptr, *sg = nullptr, *sp = nullptr;
    int e = am_ctx_scratch(s, AM_SCR_ROWS, (n + 64) * sizeof(uint32_t), &sr);
    if (!e) e = am_ctx_scratch(s, AM_SCR_GRP, 2 * (n + 64) * sizeof(uint32_t), &sg);
    if (!e) e = am_ctx_scratch(s, AM_SCR_PLAN, (n + 64) * sizeof(uint32_t), &sp);
    am_sel S;
    S.idx = idx;
    S.range = range + 2 * t;
    if (!e)
      e = run_sets_front(s, L, B, R, S, t, (uint32_t *)sp, (uint32_t *)sr, (uint32_t *)sg, ((lanes >> t) & 1u) != 0,
                         &retry[t - AM_AWSET]);
    return e;
  };
  // the planner over selection `in` (n_in reads) on c's stream, scratch slot `slot`:
  // [range: 2*NCLS][tot: NCLS][cnt: n_blk*NCLS][idx: n]
  auto plan = [&](am_ctx *c, int slot, am_sel in, uint64_t n_in, bool write_status, bool mvbig, uint32_t **range,
                  uint32_t **idx) -> int {
    const uint64_t n_blk = (n_in + PCHUNK - 1) / PCHUNK;
    void *scr = nullptr;
    if (int e = am_ctx_scratch(c, slot, (3 * NCLS + n_blk * NCLS + n + 64) * sizeof(uint32_t), &scr)) return e;
    *range = (uint32_t *)scr;
    uint32_t *tot = *range + 2 * NCLS, *cnt = tot + NCLS;
    *idx = cnt + n_blk * NCLS;
    AM_HIP(hipMemsetAsync(tot, 0, NCLS * sizeof(uint32_t), c->stream));
    hipLaunchKernelGGL(k_plan_count, dim3((unsigned)n_blk), dim3(PB), 0, c->stream, *L, *B, *R, in, cnt, tot,
                       write_status, mvbig);
    AM_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_plan_scatter, dim3((unsigned)n_blk), dim3(PB), 0, c->stream, *L, *B, *R, in, cnt, tot,
                       *range, *idx, mvbig);
    AM_HIP(hipGetLastError());
    return AM_OK;
  };
  am_sel in{};
  uint64_t n_in = n;  // reads the planner partitions
  uint32_t types = 0;
  if (lanes && (rc = log_types(ctx, L, &types))) return rc;
  // Reads whose tier is known from their key alone are planned from the whole batch and start
  // beside the lane tier: the bounded-counter chain, and the MV reads of keys in the chunked
  // big view (straight to the big-read tier; the later planner leaves them out)
  const bool bc_early = lanes && ((types >> AM_BCOUNTER) & 1u);
  // (the type mask is a per-log cache that may be stale: the log itself must hold the view)
  const bool mv_early = lanes && (types & TYPES_MVBIG) && L->key_ngrp && L->rec_g;
  uint32_t *erange = nullptr, *eidx = nullptr;
  if (lanes) {
    void *lscr = nullptr;
    rc = am_ctx_scratch(ctx, AM_SCR_SPARE, (n + 64) * sizeof(uint32_t), &lscr);
    if (rc) return rc;
    AM_HIP(hipEventRecord(ctx->ev_fork, ctx->stream));
    if (bc_early || mv_early) {
      am_ctx *es = am_ctx_sub(ctx, bc_early ? (int)(AM_BCOUNTER - AM_AWSET) : 3);
      if (!es) return AM_ERR_HIP;
      AM_HIP(hipStreamWaitEvent(es->stream, ctx->ev_fork, 0));
      rc = plan(es, AM_SCR_SPARE, all, n, false, mv_early, &erange, &eidx);
      if (!rc && mv_early) {
        ms = am_ctx_sub(ctx, 3);
        if (!ms) return AM_ERR_HIP;
        ms->grp_hint_in = ctx->grp_hint_in;
        ms->tee_a = ctx->tee_a, ms->tee_b = ctx->tee_b, ms->tee_g = ctx->tee_g, ms->tee_shift = ctx->tee_shift;
        ms->tee_done = ctx->tee_done;
        if (ms != es) {
          AM_HIP(hipEventRecord(es->ev0, es->stream));
          AM_HIP(hipStreamWaitEvent(ms->stream, es->ev0, 0));
        }
      }
      if (!rc && bc_early) rc = start_chain(AM_BCOUNTER, eidx, erange, true);
    }
    uint32_t *lbuf = (uint32_t *)lscr;  // [0] = 0, [1] = hand-off count, list at +64
    am_retry nx;
    nx.count = lbuf + 1;
    nx.list = lbuf + 64;
    if (!rc && hipMemsetAsync(lbuf, 0, 2 * sizeof(uint32_t), ctx->stream) != hipSuccess) rc = AM_ERR_HIP;
    if (!rc) rc = am_launch_lanes(ctx, L, B, R, all, nx, lanes);
    if (!rc && mv_early) {  // class 0 of the early plan: the list from 0, its count range[1]
      am_retry big;
      big.count = erange + 1;
      big.list = eidx;
      rc = am_launch_big(ms, L, B, R, AM_MVREG, big);
    }
    // one counter readback: a batch of short reads (the common case) ends here instead of
    // launching the planner and every class's kernels over empty selections
    uint64_t hc = 0;
    if (!rc) rc = am_ctx_fetch(ctx, nx.count, 1, &hc);
    n_in = (uint32_t)hc;
    if (rc || n_in == 0) {
      if (!rc && bc_early) rc = am_launch_big(sub[AM_BCOUNTER - AM_AWSET], L, B, R, AM_BCOUNTER, retry[AM_BCOUNTER - AM_AWSET]);
      join();
      return rc;
    }
    in.idx = nx.list;
    in.range = lbuf;
  }
  uint32_t *range = nullptr, *idx = nullptr;
  rc = plan(ctx, AM_SCR_PLAN, in, n_in, true, mv_early, &range, &idx);
  if (!rc && hipEventRecord(ctx->ev_fork, ctx->stream) != hipSuccess) rc = AM_ERR_HIP;
  for (uint32_t t = AM_AWSET; t <= AM_BCOUNTER && !rc; ++t)
    if (t != AM_BCOUNTER || !bc_early) rc = start_chain(t, idx, range, false);
  for (uint32_t t = AM_PN; t <= AM_LWW && !rc; ++t) {
    am_sel S;
    S.idx = idx;
    S.range = range + 2 * t;
    rc = run_scalar(ctx, L, B, R, S, t, (uint32_t *)rows_scr);
  }
  if (!rc) rc = launch_bigs_when_ready(sub, L, B, R, retry);
  join();
  return rc;
}
