// am_group.hip -- the token-group tier of the add-wins set and the MV register
// (antidote_crdt_set_aw / antidote_crdt_register_mv update/2, folded by
// clocksi_materializer:apply_operations/4, src/clocksi_materializer.erl:113-121), and the
// ingestion-side builder of the token-group view it reads (include/antidote_mat.h).
//
// Closed form.  Both types apply their effects sequentially, oldest -> newest, but the
// final state has a closed form.  Call every token an effect inserts a BIRTH at the op's
// position p (AW {Elem, [Token], _} -> (elem, token); MV {Value, Token, _} -> (value,
// token)) and every token it drops a KILL at p (AW remove tokens, MV overridden tokens).
// The AW update is ToAdd ++ (Current -- ToRemove) and the MV update drops the overridden
// tokens before insert_sorted, so a kill never hits a birth of its own op, and
//     a token survives  <=>  its newest included birth is at or after its newest included kill
// per kill key (AW (elem, token), MV token).  Tokens are unique() binaries in antidote_crdt,
// so a kill key has one birth; keys whose log breaks that (a token born twice, or under two
// MV values) are left ungrouped by the builder and go to the var_data tiers (am_sets.hip).
//
// Builder (k_grp_build, one workgroup per key, at store creation / update): the key's
// births and kills are sorted by kill key in LDS; every distinct kill key is a GROUP; the
// groups are numbered in the reference's output order -- AW: elem ascending, then newest
// birth first and, within one op, the effect's token order (ToAdd ++ Current); MV: (value,
// token) ascending (insert_sorted) -- and each birth/kill becomes one u32 record
// op | kill << 16 | group << 17.
//
// Read (k_grp_row: one 16-lane row per short read; k_grp_wave: one wave per read, up to
// 1024 groups; k_grp_wg: one 512-thread workgroup per read, up to 2048 groups):
//   1. the read's ops stream in 1024-op tiles (packed view, 16-byte loads): is_op_in_snapshot/7
//      per op (am_wave.h eval_op) -> an LDS inclusion bitmap + the scalar outputs;
//   2. the read's records (4 B each) stream in: an included birth / kill does one LDS
//      atomicMax of its op index into the group's max-birth / max-kill slot;
//   3. the groups are scanned in order: survivors (max birth >= max kill) are compacted by
//      wave ballots and their (a, b) pairs gathered into the output CSR -- already in the
//      reference's order, no sort.
// Reads with base-snapshot pairs, longer logs or ungrouped keys are handed to the next tier.
#include "am_group.h"

using namespace amk;

int am_grp_launch_d1(am_ctx *, const am_op_log *, const am_read_batch *, am_read_result *, am_sel, uint32_t, am_retry, int);
int am_grp_launch_d2(am_ctx *, const am_op_log *, const am_read_batch *, am_read_result *, am_sel, uint32_t, am_retry, int);
int am_grp_launch_d3(am_ctx *, const am_op_log *, const am_read_batch *, am_read_result *, am_sel, uint32_t, am_retry, int);
int am_grp_launch_d4(am_ctx *, const am_op_log *, const am_read_batch *, am_read_result *, am_sel, uint32_t, am_retry, int);
int am_grp_launch_d8(am_ctx *, const am_op_log *, const am_read_batch *, am_read_result *, am_sel, uint32_t, am_retry, int);
int am_grp_launch_d16(am_ctx *, const am_op_log *, const am_read_batch *, am_read_result *, am_sel, uint32_t, am_retry, int);
int am_grp_launch_d32(am_ctx *, const am_op_log *, const am_read_batch *, am_read_result *, am_sel, uint32_t, am_retry, int);

namespace {
using namespace amk_grp;


// ================================================================ builder
struct BuildSmem {
  uint64_t ka[RCAP], kb[RCAP];  // sort keys (pass 1: kill key; pass 2: output order)
  int32_t kp[RCAP];             // sort payload (pass 1: record; pass 2: raw group)
  uint32_t info[RCAP];          // per record: op index | kill << 31
  uint64_t val[RCAP], tok[RCAP];  // per record: AW elem / MV value (0 for kills), token
  uint32_t grpof[RCAP];         // per record: raw group (kill-key order)
  uint32_t bc[RCAP], bfirst[RCAP], rep[RCAP], fin[RCAP];  // per raw group
  uint32_t wsum[NW];
  uint32_t ctr[4];              // [1] outside the closed form
};

struct BuildSink {
  BuildSmem *s;
  uint32_t o, op;
  __device__ void put(uint64_t v, uint64_t t, uint32_t info) {
    if (o < RCAP) s->val[o] = v, s->tok[o] = t, s->info[o] = info;
    ++o;
  }
  __device__ void births(uint64_t e, const uint64_t *tk, uint32_t n, int32_t) {
    for (uint32_t i = 0; i < n; ++i) put(e, tk[i], op);
  }
  __device__ void birth(uint64_t a, uint64_t b, int32_t) { put(a, b, op); }
  __device__ void kills(const uint64_t *tk, uint32_t n, uint64_t e, int32_t) {
    for (uint32_t i = 0; i < n; ++i) put(e, tk[i], op | KILL31);
  }
};

// inclusive-prefix group ids over sorted positions [0, n): start flags -> ids
__device__ uint32_t raw_groups(BuildSmem &s, uint32_t n) {
  const uint32_t tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const uint64_t lt = (1ull << l) - 1ull;
  uint32_t base = 0;
  for (uint32_t c = 0; c < n; c += BLOCK) {
    const uint32_t i = c + tid;
    const bool start = i < n && (i == 0 || s.ka[i] != s.ka[i - 1] || s.kb[i] != s.kb[i - 1]);
    const uint64_t m = __ballot(start);
    if (l == 0) s.wsum[w] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t woff = 0, total = 0;
    for (int v = 0; v < NW; ++v) {
      if (v < (int)w) woff += s.wsum[v];
      total += s.wsum[v];
    }
    if (i < n) {
      const uint32_t rg = base + woff + (uint32_t)__popcll(m & lt) + (start ? 1u : 0u) - 1u;
      const uint32_t r = (uint32_t)s.kp[i];
      s.grpof[r] = rg;
      if (start) s.rep[rg] = r;
    }
    base += total;
    __syncthreads();
  }
  return base;
}

template <int TYPE>
__device__ void build_key(const am_op_log &L, BuildSmem &s, uint64_t k, uint64_t off0, uint64_t off1, uint64_t r0,
                          uint32_t n, const uint64_t *rcnt, uint32_t *rec_g, uint64_t *grp,
                          uint32_t *ngrp, uint64_t *prec) {
  const uint32_t tid = threadIdx.x;
  // 1. the key's births / kills into LDS (record order = op order, effect order within an op)
  for (uint64_t p = off0 + tid; p < off1; p += BLOCK) {
    const uint32_t meta = L.op_meta[p];
    if (meta & AM_META_BAD) continue;  // no records (k_rec_count)
    BuildSink sk{&s, (uint32_t)(rcnt[p] - r0), (uint32_t)(p - off0)};
    set_effects<TYPE>(L, p, meta, 0, sk);
  }
  if (tid == 0) s.ctr[1] = 0;
  __syncthreads();
  // 2. sort by kill key: AW (elem, token), MV token
  for (uint32_t i = tid; i < n; i += BLOCK) {
    s.ka[i] = TYPE == AM_AWSET ? s.val[i] : s.tok[i];
    s.kb[i] = TYPE == AM_AWSET ? s.tok[i] : 0ull;
    s.kp[i] = (int32_t)i;
  }
  __syncthreads();
  block_sort(s.ka, s.kb, s.kp, n, RCAP);
  const uint32_t G = raw_groups(s, n);
  // 3. births per group; the closed form needs one birth per kill key
  for (uint32_t g = tid; g < G; g += BLOCK) s.bc[g] = 0, s.bfirst[g] = 0xFFFFFFFFu;
  __syncthreads();
  for (uint32_t r = tid; r < n; r += BLOCK)
    if (!(s.info[r] & KILL31)) {
      atomicAdd(&s.bc[s.grpof[r]], 1u);
      atomicMin(&s.bfirst[s.grpof[r]], r);
    }
  __syncthreads();
  for (uint32_t r = tid; r < n; r += BLOCK)
    if (!(s.info[r] & KILL31)) {
      const uint32_t g = s.grpof[r];
      if (s.bc[g] > 1) s.ctr[1] = 1;  // a token born twice (AW) / twice or under two values (MV)
    }
  __syncthreads();
  if (s.ctr[1]) {
    if (tid == 0) ngrp[k] = AM_NGRP_NONE;
    __syncthreads();
    return;
  }
  // 4. groups in output order.  AW: elem, then the newest birth op first, then the
  //    effect's token order (record index); MV: (value, token).  Unborn groups last.
  for (uint32_t g = tid; g < G; g += BLOCK) {
    const uint32_t b = s.bfirst[g], rp = s.rep[g];
    const bool born = b != 0xFFFFFFFFu;
    if (TYPE == AM_AWSET) {
      s.ka[g] = s.val[rp];
      s.kb[g] = born ? (((uint64_t)(0x7FFFFFFFu - (s.info[b] & 0xFFFFu)) << 32) | b) : ~0ull;
    } else {
      s.ka[g] = born ? s.val[b] : ~0ull;
      s.kb[g] = s.tok[rp];
    }
    s.kp[g] = (int32_t)g;
  }
  __syncthreads();
  block_sort(s.ka, s.kb, s.kp, G, RCAP);
  for (uint32_t j = tid; j < G; j += BLOCK) {
    const uint32_t rg = (uint32_t)s.kp[j];
    s.fin[rg] = j;
    grp[2 * (r0 + j)] = s.ka[j];  // AW elem; MV value (~0: no birth)
    grp[2 * (r0 + j) + 1] = TYPE == AM_AWSET ? s.tok[s.rep[rg]] : s.kb[j];
  }
  __syncthreads();
  // records; a kill of a born group is EFFECTIVE only after the birth (a kill in the birth's
  // own op or before it never removes the token): the others become empty slots
  // (0xFFFFFFFF).  Kills of a group with no birth in the log are kept: such a group is never
  // output from the log alone, but a cached base snapshot may hold its token (born by an op
  // pruned since), which an included kill removes (k_grp_wave's base merge)
  for (uint32_t r = tid; r < n; r += BLOCK) {
    const uint32_t g = s.grpof[r], b = s.bfirst[g];
    const uint32_t op = s.info[r] & 0xFFFFu;
    const bool kill = (s.info[r] & KILL31) != 0;
    const bool keep = !kill || b == 0xFFFFFFFFu || op > (s.info[b] & 0xFFFFu);
    rec_g[r0 + r] = keep ? (op | ((kill ? 1u : 0u) << 16) | (s.fin[g] << 17)) : 0xFFFFFFFFu;
    if (prec && !kill) {  // a birth's (elem | value, token) is its group's pair
      prec[2 * (r0 + r)] = s.val[r];
      prec[2 * (r0 + r) + 1] = s.tok[r];
    }
  }
  if (tid == 0) ngrp[k] = G;
  __syncthreads();
}

__global__ void __launch_bounds__(BLOCK) k_grp_build(am_op_log L, const uint64_t *rcnt, uint32_t *rec_g, uint64_t *grp,
                                                     uint32_t *ngrp, uint64_t *prec) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  BuildSmem &s = *reinterpret_cast<BuildSmem *>(smem_raw);
  for (uint64_t k = blockIdx.x; k < L.n_keys; k += gridDim.x) {
    const uint32_t type = uniform_u32(L.key_type[k]);
    const uint32_t kfl = L.key_flags ? uniform_u32(L.key_flags[k]) : 0u;
    const uint64_t off0 = uniform_u64(L.key_off[k]), off1 = uniform_u64(am_kend(L, k));
    const uint64_t r0 = uniform_u64(rcnt[off0]), r1 = uniform_u64(rcnt[off1]);
    const uint64_t n = r1 - r0;
    const bool set = type == AM_AWSET || type == AM_MVREG;
    if (!set || n > RCAP || off1 - off0 >= 65536 || (kfl & AM_KEY_MIXED_TYPES) || am_big_grp_key(L, k)) {
      if (threadIdx.x == 0) ngrp[k] = AM_NGRP_NONE;
      continue;
    }
    if (type == AM_AWSET) build_key<AM_AWSET>(L, s, k, off0, off1, r0, (uint32_t)n, rcnt, rec_g, grp, ngrp, prec);
    else build_key<AM_MVREG>(L, s, k, off0, off1, r0, (uint32_t)n, rcnt, rec_g, grp, ngrp, prec);
  }
}

}  // namespace

bool am_group_applies(const am_op_log *L, const am_read_result *R, uint32_t type) {
  return (type == AM_AWSET || type == AM_MVREG) && L->rec_key_off && L->rec_g && L->grp && L->key_ngrp &&
         L->op_meta && R->value.set_off && R->value.set_len && R->value.set_a && R->value.set_b;
}

int am_launch_group(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S,
                    uint32_t type, am_retry next, int tier) {
  const uint32_t nd = L->n_dc;
  if (nd <= 1) return am_grp_launch_d1(ctx, L, B, R, S, type, next, tier);
  if (nd <= 2) return am_grp_launch_d2(ctx, L, B, R, S, type, next, tier);
  if (nd <= 3) return am_grp_launch_d3(ctx, L, B, R, S, type, next, tier);
  if (nd <= 4) return am_grp_launch_d4(ctx, L, B, R, S, type, next, tier);
  if (nd <= 8) return am_grp_launch_d8(ctx, L, B, R, S, type, next, tier);
  if (nd <= 16) return am_grp_launch_d16(ctx, L, B, R, S, type, next, tier);
  return am_grp_launch_d32(ctx, L, B, R, S, type, next, tier);
}

int am_launch_group_build(am_ctx *ctx, const am_op_log *L, const uint64_t *rcnt, uint32_t *rec_g, uint64_t *grp,
                          uint32_t *key_ngrp, uint64_t *prec) {
  if (L->n_keys == 0) return AM_OK;
  constexpr size_t smem = sizeof(BuildSmem);
  static bool attr = false;
  if (!attr) {
    AM_HIP(hipFuncSetAttribute((const void *)k_grp_build, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
    attr = true;
  }
  const uint64_t blocks = L->n_keys < (uint64_t)ctx->n_cu * 8 ? L->n_keys : (uint64_t)ctx->n_cu * 8;
  hipLaunchKernelGGL(k_grp_build, dim3((unsigned)blocks), dim3(BLOCK), smem, ctx->stream, *L, rcnt, rec_g, grp,
                     key_ngrp, prec);
  AM_HIP(hipGetLastError());
  return AM_OK;
}
