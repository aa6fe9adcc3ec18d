// am_bcrows.hip -- materialize/4 for SHORT bounded-counter reads (antidote_crdt_counter_b:
// orddict:update_counter on P[{From,To}] and D[Id] is a keyed sum, folded by
// clocksi_materializer:apply_operations/4, src/clocksi_materializer.erl:113-121), batch clock,
// packed view, n_dc <= 16: one 16-lane row per read, four reads of a wave at a time.
//
// The general row tier (am_rows.hip) keeps a read's D*D + D slot sums in an LDS array: every
// read clears all 272 slots (D = 16), adds each included amount with a 64-bit LDS atomic and
// scans the array to emit -- for reads averaging a few dozen ops that touch a handful of slots --
// and its full-width per-DC state holds it at one wave per SIMD.  Here a read's result is built
// from the slots it touches only:
//   * each lane evaluates up to 4 ops (16-op steps; is_op_in_snapshot/7 on the packed u32
//     entries against thresholds computed once per read) and keeps its included ops' (slot,
//     amount) pairs in registers;
//   * the row marks the touched slots in a 272-bit LDS bitmap (one atomicOr per included op):
//     the slot's rank among the touched ones is its place in the orddicts' key order (P
//     {From,To} then D Id), so the result needs no sort;
//   * the amounts are summed at their rank in a compact LDS array (<= 64 entries, exact: every
//     |amount| < 2^56, a larger one defers the read), and lane l emits entries l, l + 16, ...:
//     its slot is the rank's set bit of the bitmap, its value the sum;
//   * LastOpCt entries are u32 maxima relative to the key's time base (row DPP reductions),
//     written by lane d of the row; the scalar outputs go through LDS to the read's lane and
//     leave with one coalesced store per column.
// Ops outside the packed view are evaluated from the full columns by the row, one DC per lane.
// Reads it does not take (> BCR_OPS ops) go to `next`.
#include "am_block.h"

using namespace amk;

namespace {

constexpr int BLOCK = 256;
constexpr int RG = 16;              // lanes per row
constexpr uint32_t BCR_OPS = 64;    // 4 steps of 16 ops
constexpr uint32_t NSW = 9;         // bitmap words: 16 * 16 + 16 = 272 slots

struct BcrIn {  // a taken read of the batch, for the row that reads it
  uint64_t off0, K, idb, ooff;
  uint32_t nops, cap, r, tk;
};
struct BcrOut {  // its scalar outputs, for the read's lane
  int64_t nlo;
  int32_t status;
  uint32_t flags, count, nent, pres;
  uint32_t store;  // 0: deferred to the next tier
};
struct BcrRow {
  uint32_t bm[NSW + 1];  // + a defer flag
  int64_t sum[BCR_OPS];
};
struct BcrSmem {
  BcrIn in[WAVE];
  BcrOut out[WAVE];
  BcrRow row[WAVE / RG];
};

__device__ __forceinline__ uint32_t row_min_u32(uint32_t v) {
#define S_(C) v = min(v, dpp32<C>(v));
  AMK_ROW_STEPS(S_)
#undef S_
  return v;
}
__device__ __forceinline__ uint32_t row_max_u32(uint32_t v) {
#define S_(C) v = max(v, dpp32<C>(v));
  AMK_ROW_STEPS(S_)
#undef S_
  return v;
}

template <int DMAX>
__global__ void __launch_bounds__(BLOCK) k_bc_rows(am_op_log L, am_read_batch B, am_read_result R, am_sel S,
                                                   am_retry next) {
  __shared__ BcrSmem smem[BLOCK / WAVE];
  BcrSmem &sm = smem[threadIdx.x / WAVE];
  const uint32_t lane = threadIdx.x & (WAVE - 1), row = lane / RG, sl = lane % RG;
  const uint64_t lt = (1ull << lane) - 1ull;
  BcrRow &rs = sm.row[row];
  const uint32_t nd = L.n_dc, np = nd * nd;
  const uint64_t n = B.n_reads;
  const uint64_t stride = L.snap_stride ? L.snap_stride : L.n_ops;
  const uint32_t sel0 = S.idx ? uniform_u32(S.range[0]) : 0u;
  const uint64_t nsel = S.idx ? (uint64_t)(uniform_u32(S.range[1]) - sel0) : n;
  const uint64_t W = (uint64_t)gridDim.x * (BLOCK / WAVE);
  const uint64_t gw = (uint64_t)blockIdx.x * (BLOCK / WAVE) + uniform_u32(threadIdx.x >> 6);
  ReadU<DMAX> u{};
  {  // the batch clock (base ignore, no TxIds)
    u.allmask = nd >= 32 ? 0xFFFFFFFFu : ((1u << nd) - 1u);
    u.spres = uniform_u32(B.read_pres[0]) & u.allmask;
    u.base_ignore = true;
#pragma unroll
    for (int d = 0; d < DMAX; ++d) u.S[d] = (d < (int)nd && ((u.spres >> d) & 1u)) ? uniform_u64(B.read_vc[d]) : 0;
  }
  const uint32_t miss = (u.allmask & ~u.spres) ? AM_FLAG_MISSING_DC_LOGGED : 0u;

  for (uint64_t rb = gw * WAVE; rb < nsel; rb += W * WAVE) {
    // ---- lane i: read rb + i -> status | hand-off | taken (published for its row) ----
    const uint64_t i = rb + lane;
    bool take = false, hand = false;
    uint64_t r = 0;
    if (i < nsel) {
      r = S.idx ? (uint64_t)S.idx[sel0 + i] : i;
      const uint64_t key = B.key[r];
      int32_t st = AM_OK;
      uint64_t off0 = 0, off1 = 0;
      if (key >= L.n_keys) {
        st = AM_ERR_INVALID;
      } else {
        off0 = L.key_off[key];
        off1 = am_kend(L, key);
        const uint32_t ktype = L.key_type[key], kfl = L.key_flags ? (uint32_t)L.key_flags[key] : 0u;
        if (off1 > off0 && (ktype != (uint32_t)B.type[r] || (kfl & AM_KEY_MIXED_TYPES))) st = AM_ERR_CORRUPTED_OPS_CACHE;
        else if (B.type[r] != AM_BCOUNTER) st = AM_ERR_INVALID;
      }
      if (st != AM_OK) {
        R.status[r] = st, R.flags[r] = 0;
      } else if (off1 - off0 > BCR_OPS) {
        hand = true;
      } else {
        take = true;
        BcrIn &w = sm.in[lane];
        w.off0 = off0, w.nops = (uint32_t)(off1 - off0), w.K = L.key_tbase[key];
        w.idb = L.key_id_base ? L.key_id_base[key] : 1;
        w.ooff = R.value.set_off[r];
        const uint64_t cap = R.value.set_off[r + 1] - w.ooff;
        w.cap = cap < 0xFFFFFFFFull ? (uint32_t)cap : 0xFFFFFFFFu;
        w.r = (uint32_t)r;
      }
      sm.out[lane].store = 0;
    }
    sm.in[lane].tk = take ? 1u : 0u;
    const uint64_t hm = __ballot(hand);
    if (hm) {
      uint32_t base = 0;
      if (lane == 0) base = atomicAdd(next.count, (uint32_t)__popcll(hm));
      base = uniform_u32(base);
      if (hand) next.list[base + (uint32_t)__popcll(hm & lt)] = (uint32_t)r;
    }
    const uint64_t tm = __ballot(take);
    wave_sync();

    // ---- row q reads the batch's reads q, q + 4, ... (every row in lockstep, full EXEC).  The
    //      first 16 ops of the row's next read are loaded while this one is evaluated (most
    //      reads have at most 16) ----
    uint32_t nx[DMAX], nmeta = 0;
    int64_t namt = 0;
    uint64_t nft = 0;
    auto load_op = [&](const BcrIn &w, uint32_t q, uint32_t(&x)[DMAX], uint32_t &meta, int64_t &amt, uint64_t &ft) {
      const uint64_t p = (w.tk && q < w.nops) ? w.off0 + q : 0;  // (a row without a read loads op 0, unused)
#pragma unroll
      for (int d = 0; d < DMAX; ++d) x[d] = d < (int)nd ? L.pk_vc[(uint64_t)d * stride + p] : 0u;
      meta = L.op_meta[p], amt = (int64_t)L.p0[p], ft = L.p1[p];
    };
    if (tm) load_op(sm.in[row], sl, nx, nmeta, namt, nft);
    for (uint32_t it = 0; it < WAVE / 4 && (tm >> (4 * it)); ++it) {
      const uint32_t j = 4 * it + row;
      const BcrIn in = sm.in[j];
      uint32_t cx[DMAX];
#pragma unroll
      for (int d = 0; d < DMAX; ++d) cx[d] = nx[d];
      const uint32_t cmeta = nmeta;
      const int64_t camt = namt;
      const uint64_t cft = nft;
      if (it + 1 < WAVE / 4 && (tm >> (4 * (it + 1)))) load_op(sm.in[j + 4], sl, nx, nmeta, namt, nft);
      const bool act = in.tk != 0;
      PkRead<DMAX> pk;
      pk_setup(u, nd, in.K, pk);
      if (sl < NSW + 1) rs.bm[sl] = 0;
      wave_sync();
      uint32_t mx[DMAX];
#pragma unroll
      for (int d = 0; d < DMAX; ++d) mx[d] = 0;
      uint32_t cnt = 0, fl = 0, mex = 0xFFFFFFFFu, esc = 0;
      uint32_t pslot[BCR_OPS / RG];
      int64_t pamt[BCR_OPS / RG];
      uint32_t pv = 0;  // pairs held
#pragma unroll
      for (uint32_t t = 0; t < BCR_OPS / RG; ++t) {
        pslot[t] = 0, pamt[t] = 0;
        if (!__ballot(act && RG * t < in.nops)) continue;
        const uint32_t q = RG * t + sl;
        const bool v = act && q < in.nops;
        uint32_t x[DMAX], meta;
        int64_t amt;
        uint64_t ft;
        if (t == 0) {  // prefetched
#pragma unroll
          for (int d = 0; d < DMAX; ++d) x[d] = cx[d];
          meta = cmeta, amt = camt, ft = cft;
        } else {
          load_op(in, q, x, meta, amt, ft);
        }
        if (!v) continue;
        if (x[0] == AM_PK_ESC) {  // outside the packed view: the row evaluates it below
          esc |= 1u << t;
          continue;
        }
        uint32_t over = 0;
#pragma unroll
        for (int d = 0; d < DMAX; ++d) over |= __builtin_elementwise_sub_sat(x[d], pk.thr[d]);
        fl |= pk.miss;
        if (pk.never || over) {
          mex = min(mex, q);
          continue;
        }
#pragma unroll
        for (int d = 0; d < DMAX; ++d) mx[d] = max(mx[d], x[d]);
        ++cnt;
        const uint32_t kind = AM_META_KIND(meta), from = (uint32_t)(ft & 0xFF), to = (uint32_t)((ft >> 8) & 0xFF);
        if (kind > AM_BC_TRANSFER || from >= nd || to >= nd) {  // Type:update/2 would raise
          fl |= FLAG_BAD;
          continue;
        }
        const uint32_t slot = kind == AM_BC_DECREMENT ? np + from : from * nd + (kind == AM_BC_INCREMENT ? from : to);
        if (amt >= (1ll << 56) || amt < -(1ll << 56)) rs.bm[NSW] = 1;  // exactness of the int64 sums: defer
        atomicOr(&rs.bm[slot >> 5], 1u << (slot & 31));
        pslot[t] = slot, pamt[t] = amt, pv |= 1u << t;
      }
      // ops outside the packed view, one at a time by the whole row (lane d: DC d)
      uint64_t emx = 0;   // lane d: the max X[d] of the included escaped ops
      uint32_t ecnt = 0;  // (row-uniform)
      for (uint32_t lm = row_or_u32(esc ? 1u << sl : 0u); lm; lm &= lm - 1) {
        const uint32_t owner = (uint32_t)__builtin_ctz(lm);
        for (uint32_t tb = shfl_u32(esc, row * RG + owner); tb; tb &= tb - 1) {
          const uint32_t t = (uint32_t)__builtin_ctz(tb), q = RG * t + owner;
          const uint64_t p = in.off0 + q;
          const uint64_t *w = esc_row(L, stride, p);  // its escape row, or the columns
          const uint32_t meta = w ? (uint32_t)w[1] : L.op_meta[p], dc = meta & 31u;
          uint64_t xd = 0, sd = 0;
          if (sl < nd) xd = sl == dc ? (w ? w[0] : L.commit_time[p]) : (w ? w[2 + sl] : L.snap_vc[(uint64_t)sl * stride + p]);
#pragma unroll
          for (int d = 0; d < DMAX; ++d)
            if ((uint32_t)d == sl) sd = u.S[d];
          const bool fail = sl < nd && (!((u.spres >> sl) & 1u) || xd > sd);
          const bool included = row_or_u32(fail ? 1u : 0u) == 0;
          if (sl == 0) fl |= miss;
          if (!included) {
            if (sl == 0) mex = min(mex, q);
            continue;
          }
          emx = max(emx, xd);
          ++ecnt;
          if (sl != owner) continue;  // the op's lane applies its effect
          if (meta & AM_META_BAD) {
            fl |= FLAG_BAD;
            continue;
          }
          const int64_t amt = (int64_t)L.p0[p];
          const uint64_t ft = L.p1[p];
          const uint32_t kind = AM_META_KIND(meta), from = (uint32_t)(ft & 0xFF), to = (uint32_t)((ft >> 8) & 0xFF);
          if (kind > AM_BC_TRANSFER || from >= nd || to >= nd) {
            fl |= FLAG_BAD;
            continue;
          }
          const uint32_t slot = kind == AM_BC_DECREMENT ? np + from : from * nd + (kind == AM_BC_INCREMENT ? from : to);
          if (amt >= (1ll << 56) || amt < -(1ll << 56)) rs.bm[NSW] = 1;
          atomicOr(&rs.bm[slot >> 5], 1u << (slot & 31));
#pragma unroll
          for (uint32_t tt = 0; tt < BCR_OPS / RG; ++tt)
            if (tt == t) pslot[tt] = slot, pamt[tt] = amt;
          pv |= 1u << t;
        }
      }
      wave_sync();
      // ---- the touched slots: ranks in key order; compact sums ----
      uint32_t bm[NSW], below[NSW], ns = 0;
#pragma unroll
      for (uint32_t w = 0; w < NSW; ++w) bm[w] = rs.bm[w], below[w] = ns, ns += (uint32_t)__popc(bm[w]);
      const bool defer = act && rs.bm[NSW] != 0;
      for (uint32_t e = sl; e < ns; e += RG) rs.sum[e] = 0;
      wave_sync();
#pragma unroll
      for (uint32_t t = 0; t < BCR_OPS / RG; ++t) {
        if (!((pv >> t) & 1u)) continue;
        const uint32_t s = pslot[t], w = s >> 5;
        uint32_t rank = 0;
#pragma unroll
        for (uint32_t k = 0; k < NSW; ++k)
          if (k == w) rank = below[k] + (uint32_t)__popc(bm[k] & ((1u << (s & 31)) - 1u));
        atomicAdd((unsigned long long *)&rs.sum[rank], (unsigned long long)pamt[t]);
      }
      wave_sync();
      // ---- row reductions (full EXEC) ----
      const uint32_t count = row_sum_u32(cnt) + ecnt;
      const uint32_t flags = row_or_u32(fl);
      const uint32_t minq = row_min_u32(mex);
      uint64_t myct = 0;  // lane d: LastOpCt entry d (max X[d] of the included ops)
#pragma unroll
      for (int d = 0; d < DMAX; ++d) {
        if (d >= (int)nd) continue;
        const uint32_t m = row_max_u32(mx[d]);
        if ((uint32_t)d == sl) myct = (count - ecnt) ? in.K + m : 0;
      }
      myct = max(myct, emx);
      int32_t status = (flags & FLAG_BAD) ? AM_ERR_UNEXPECTED_OPERATION : AM_OK;
      uint32_t nent = 0;
      if (act && !defer && status == AM_OK) {  // the touched slots as (slot, value) pairs
        nent = ns;
        for (uint32_t e = sl; e < ns && e < in.cap; e += RG) {
          uint32_t w = 0, k = e;  // the e-th set bit of the bitmap
#pragma unroll
          for (uint32_t x = 0; x < NSW; ++x)
            if (e >= below[x] && e < below[x] + (uint32_t)__popc(bm[x])) w = x, k = e - below[x];
          uint32_t bits = bm[w];
          for (uint32_t c = 0; c < k; ++c) bits &= bits - 1;
          R.value.set_a[in.ooff + e] = 32 * w + (uint32_t)__builtin_ctz(bits);
          R.value.set_b[in.ooff + e] = (uint64_t)rs.sum[e];
        }
        if (ns > in.cap) status = AM_ERR_CAPACITY;
      }
      const bool ign = count == 0;  // base ignore: LastOpCt = ignore without included ops
      const uint32_t opres = ign ? 0u : u.allmask;
      if (act && !defer && status == AM_OK && sl < nd) R.last_ct[(uint64_t)sl * n + in.r] = myct;
      if (act && sl == 0) {
        if (defer) next.list[atomicAdd(next.count, 1u)] = in.r;
        BcrOut &o = sm.out[j];
        o.store = defer ? 0u : 1u;
        o.status = status, o.flags = flags & 0xFFu, o.count = count, o.nent = nent, o.pres = opres;
        o.nlo = minq != 0xFFFFFFFFu ? (int64_t)(in.idb + minq) - 1
                                    : (in.nops == 0 ? 0 : (int64_t)(in.idb + in.nops - 1));
      }
      wave_sync();
    }
    // ---- the batch's outputs: one coalesced store per column ----
    if ((tm >> lane) & 1u) {
      const BcrOut o = sm.out[lane];
      if (o.store) {
        R.status[r] = o.status;
        R.flags[r] = (uint8_t)o.flags;
        if (o.status == AM_OK) {
          R.new_last_op[r] = o.nlo;
          R.last_ct_ignore[r] = o.count == 0 ? 1 : 0;
          R.last_ct_pres[r] = o.pres;
          R.is_new_ss[r] = o.count > 0;
          R.count[r] = o.count;
          R.value.set_len[r] = o.nent;
        }
      }
    }
    wave_sync();  // the LDS areas are rewritten by the next batch
  }
}

template <int D>
int launch_d(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S, am_retry next) {
  static int occ = 0;
  if (!occ && (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_bc_rows<D>, BLOCK, 0) != hipSuccess || occ < 1))
    occ = 1;
  const uint64_t batches = (B->n_reads + WAVE - 1) / WAVE;
  uint64_t blocks = (batches + BLOCK / WAVE - 1) / (BLOCK / WAVE), cap = (uint64_t)ctx->n_cu * occ;
  if (blocks > cap) blocks = cap;
  if (blocks == 0) return AM_OK;
  hipLaunchKernelGGL((k_bc_rows<D>), dim3((unsigned)blocks), dim3(BLOCK), 0, ctx->stream, *L, *B, *R, S, next);
  AM_HIP(hipGetLastError());
  return AM_OK;
}

}  // namespace

// the batch clock, packed view, n_dc <= 16, no op ids / TxIds / bases, the sparse value CSR
bool am_bcrows_applies(const am_op_log *L, const am_read_batch *B, const am_read_result *R) {
  return am_log_packed(L) && !am_batch_general(L, B) && L->n_dc <= 16 && L->op_meta && R->value.set_off &&
         R->value.set_len && R->value.set_a && R->value.set_b;
}

int am_launch_bcrows(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S,
                     am_retry next) {
  const uint32_t nd = L->n_dc;
  if (nd <= 1) return launch_d<1>(ctx, L, B, R, S, next);
  if (nd <= 2) return launch_d<2>(ctx, L, B, R, S, next);
  if (nd <= 3) return launch_d<3>(ctx, L, B, R, S, next);
  if (nd <= 4) return launch_d<4>(ctx, L, B, R, S, next);
  if (nd <= 8) return launch_d<8>(ctx, L, B, R, S, next);
  return launch_d<16>(ctx, L, B, R, S, next);
}
