// am_bcrows.hip -- materialize/4 for SHORT bounded-counter reads (antidote_crdt_counter_b:
// orddict:update_counter on P[{From,To}] and D[Id] is a keyed sum, folded by
// clocksi_materializer:apply_operations/4, src/clocksi_materializer.erl:113-121), batch clock,
// packed or lag view, n_dc <= 16: one 16-lane row per read, four reads of a wave at a time.
//
// The general row tier (am_rows.hip) keeps a read's D*D + D slot sums in an LDS array: every
// read clears all 272 slots (D = 16), adds each included amount with a 64-bit LDS atomic and
// scans the array to emit -- for reads averaging a few dozen ops that touch a handful of slots --
// and its full-width per-DC state holds it at one wave per SIMD.  Here a read's result is built
// from the slots it touches only:
//   * lane d of the row holds DC d: a step takes a 16-op window aligned to 4 and loads DC d's
//     entries of it (four 16-byte loads of the packed view; at D > 8 the lag view: DC d's u16
//     lags, the commit words shared by the row), so is_op_in_snapshot/7 is one row OR of the
//     lanes' fail bits per window and lane d's LastOpCt entry is its own running maximum (u32,
//     relative to the key's time base, no reductions);
//   * lane k applies op k of the window: the row marks the touched slots in a 272-bit LDS bitmap
//     (one atomicOr per included op) and keeps its (slot, amount) pairs in registers; the slot's
//     rank among the touched ones is its place in the orddicts' key order (P {From,To} then
//     D Id), so the result needs no sort;
//   * the amounts are summed at their rank in a compact LDS array (<= 64 entries, exact: every
//     |amount| < 2^56, a larger one defers the read), and lane l emits entries l, l + 16, ...:
//     its slot is the rank's set bit of the bitmap, its value the sum;
//   * the scalar outputs go through LDS to the read's lane and leave with one coalesced store
//     per column; the next read's first window is loaded while a read is evaluated.
// Ops outside the views are evaluated from their escape rows or the full columns by the row,
// one DC per lane.  Reads it does not take (> BCR_OPS ops) go to `next`.
#include "am_block.h"

using namespace amk;

namespace {

constexpr int BLOCK = 256;
constexpr int RG = 16;              // lanes per row
constexpr uint32_t BCR_OPS = 64;    // 4 steps of 16 ops
constexpr uint32_t NSW = 9;         // bitmap words: 16 * 16 + 16 = 272 slots

struct BcrIn {  // a taken read of the batch, for the row that reads it
  uint64_t off0, K, idb, ooff, key;
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

#ifndef AM_BCR_PREFETCH
#define AM_BCR_PREFETCH 1  // the next read's first window loaded while this read is evaluated
#endif
#ifndef AM_BCR_WAVES
#define AM_BCR_WAVES 1     // waves per SIMD the kernel is compiled for (1: the compiler's choice)
#endif
template <int DMAX, bool LAG>
__global__ void __launch_bounds__(BLOCK, AM_BCR_WAVES) k_bc_rows(am_op_log L, am_read_batch B, am_read_result R, am_sel S,
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
        w.r = (uint32_t)r, w.key = key;
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

    // ---- row q reads the batch's reads q, q + 4, ... (every row in lockstep, full EXEC).  Lane
    //      d of a row holds DC d: a step takes a 16-op window aligned to 4 (four 16-byte loads of
    //      the DC's packed entries), the window's failures are one row OR of the lanes' fail
    //      bits, and lane d's LastOpCt entry is its own running maximum.  Lane k applies op k of
    //      the window.  The next read's first window is loaded while this read is evaluated ----
    uint64_t vS = 0;  // lane d: the clock entry S[d]
#pragma unroll
    for (int d = 0; d < DMAX; ++d) vS = (uint32_t)d == sl ? u.S[d] : vS;
    const bool dl = sl < nd;  // the lane holds a DC of the log
    struct Win {
      u32x4 e[4];  // DC sl's packed entries of the window's ops 0..15 (LAG: the ops' lag_ct)
      uint2 g[4];  // LAG: DC sl's u16 lags of the window's ops
      uint32_t lb;  // LAG: the key's lag base of DC sl (the read's first window)
      uint32_t meta;
      int64_t amt;
      uint64_t ft;  // op sl of the window
    };
    auto load_win = [&](const BcrIn &w, uint32_t t, Win &x) {
      const uint64_t wb = (w.off0 & ~3ull) + (uint64_t)RG * t, end = w.off0 + w.nops;
      const bool any = w.tk != 0 && wb < end;
      // unpredicated: a quad the read does not need (or a pad lane's) is loaded from the
      // column's first line and ignored
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        if constexpr (LAG) {  // 4 + 2 D bytes per op: the row shares the lag_ct lines
          const bool in = any && wb + 4 * h < end;
          x.e[h] = *(const u32x4 *)(L.lag_ct + (in ? wb + 4 * h : 0));
          x.g[h] = *(const uint2 *)(L.lag + ((in && dl) ? (uint64_t)sl * stride + wb + 4 * h : 0));
        } else {
          const uint64_t a = (any && dl && wb + 4 * h < end) ? (uint64_t)sl * stride + wb + 4 * h : 0;
          x.e[h] = *(const u32x4 *)(L.pk_vc + a);
        }
      }
      if (LAG && t == 0) x.lb = (w.tk != 0 && dl) ? (uint32_t)L.key_lag[w.key * nd + sl] : 0u;
      const uint64_t p = wb + sl;
      const uint64_t pp = (any && p >= w.off0 && p < end) ? p : 0;
      x.meta = L.op_meta[pp], x.amt = (int64_t)L.p0[pp], x.ft = L.p1[pp];
    };
    constexpr uint32_t NST = BCR_OPS / RG + 1;  // windows of a read of <= 64 ops from off0 & ~3
    Win nx;
    if (AM_BCR_PREFETCH && tm) load_win(sm.in[row], 0, nx);
    for (uint32_t it = 0; it < WAVE / 4 && (tm >> (4 * it)); ++it) {
      const uint32_t j = 4 * it + row;
      const BcrIn in = sm.in[j];
      const Win cx = nx;
      const uint32_t lb = LAG ? cx.lb : 0u;  // this read's lag base of DC sl
      if (AM_BCR_PREFETCH && it + 1 < WAVE / 4 && (tm >> (4 * (it + 1)))) load_win(sm.in[j + 4], 0, nx);
      const bool act = in.tk != 0;
      const uint64_t a0 = in.off0 & ~3ull, end = in.off0 + in.nops;
      const uint32_t thr = dl ? pk_clamp(vS, in.K) : AM_PK_ESC;  // pad lanes pass
      const bool never = miss != 0 || row_or_u32((dl && vS < in.K) ? 1u : 0u) != 0;
      if (sl < NSW + 1) rs.bm[sl] = 0;
      wave_sync();
      uint32_t mxl = 0;  // lane d: max X[d] - K of the included ops (packed)
      uint32_t cnt = 0, fl = 0, mex = 0xFFFFFFFFu, esc = 0;  // cnt, mex: row-uniform
      uint32_t pslot[NST];
      int64_t pamt[NST];
      uint32_t pv = 0;  // pairs held (bit t: op sl of window t)
#pragma unroll
      for (uint32_t t = 0; t < NST; ++t) {
        pslot[t] = 0, pamt[t] = 0;
        const uint64_t wb = a0 + (uint64_t)RG * t;
        if (!__ballot(act && wb < end)) continue;
        Win x;
        if (AM_BCR_PREFETCH && t == 0) x = cx;  // prefetched
        else load_win(in, t, x);
        uint32_t ob = 0, eb = 0;  // the lane's fail bits; escape marks (lane 0: DC 0 == AM_PK_ESC)
        if constexpr (LAG) {  // X[d] - K = lag_ct - (key_lag[d] + lag[d]); escapes: lag_ct == AM_PK_ESC
#pragma unroll
          for (int k = 0; k < 16; ++k) {
            const uint32_t c = x.e[k >> 2][k & 3], gw = (k & 2) ? x.g[k >> 2].y : x.g[k >> 2].x;
            const uint32_t e = c - (lb + ((k & 1) ? gw >> 16 : gw & 0xFFFFu));
            x.e[k >> 2][k & 3] = e;
            ob |= (uint32_t)(e > thr) << k;
            eb |= (uint32_t)(c == AM_PK_ESC) << k;
          }
        } else {
#pragma unroll
          for (int k = 0; k < 16; ++k) {
            const uint32_t e = x.e[k >> 2][k & 3];
            ob |= (uint32_t)(e > thr) << k;
            eb |= (uint32_t)(e == AM_PK_ESC) << k;
          }
        }
        const uint32_t fail = row_or_u32(ob);
        const uint32_t em = LAG ? eb : shfl_u32(eb, row * RG);
        uint32_t vm = 0;  // the window's ops inside [off0, off1)
        if (act && wb < end) {
          const uint32_t lo = in.off0 > wb ? (uint32_t)(in.off0 - wb) : 0u;
          const uint32_t hi = end - wb < (uint64_t)RG ? (uint32_t)(end - wb) : RG;
          vm = ((1u << hi) - 1u) & ~((1u << lo) - 1u);
        }
        const uint32_t cand = vm & ~em, inc = never ? 0u : cand & ~fail;
        if (cand) fl |= miss;
        cnt += (uint32_t)__popc(inc);
        const uint32_t ex = cand & ~inc;
        if (ex) mex = min(mex, (uint32_t)(wb - in.off0) + (uint32_t)__builtin_ctz(ex));
#pragma unroll
        for (int k = 0; k < 16; ++k) mxl = max(mxl, ((inc >> k) & 1u) ? x.e[k >> 2][k & 3] : 0u);
        if (((vm & em) >> sl) & 1u) esc |= 1u << t;  // op sl escaped: the row evaluates it below
        if (!((inc >> sl) & 1u)) continue;
        const uint32_t kind = AM_META_KIND(x.meta), from = (uint32_t)(x.ft & 0xFF), to = (uint32_t)((x.ft >> 8) & 0xFF);
        if (kind > AM_BC_TRANSFER || from >= nd || to >= nd) {  // Type:update/2 would raise
          fl |= FLAG_BAD;
          continue;
        }
        const uint32_t slot = kind == AM_BC_DECREMENT ? np + from : from * nd + (kind == AM_BC_INCREMENT ? from : to);
        if (x.amt >= (1ll << 56) || x.amt < -(1ll << 56)) rs.bm[NSW] = 1;  // exactness of the int64 sums: defer
        atomicOr(&rs.bm[slot >> 5], 1u << (slot & 31));
        pslot[t] = slot, pamt[t] = x.amt, pv |= 1u << t;
      }
      // ops outside the packed view, one at a time by the whole row (lane d: DC d)
      uint64_t emx = 0;   // lane d: the max X[d] of the included escaped ops
      uint32_t ecnt = 0;  // (row-uniform)
      for (uint32_t lm = row_or_u32(esc ? 1u << sl : 0u); lm; lm &= lm - 1) {
        const uint32_t owner = (uint32_t)__builtin_ctz(lm);
        for (uint32_t tb = shfl_u32(esc, row * RG + owner); tb; tb &= tb - 1) {
          const uint32_t t = (uint32_t)__builtin_ctz(tb);
          const uint64_t p = a0 + (uint64_t)RG * t + owner;
          const uint32_t q = (uint32_t)(p - in.off0);
          const uint64_t *w = esc_row(L, stride, p);  // its escape row, or the columns
          const uint32_t meta = w ? (uint32_t)w[1] : L.op_meta[p], dc = meta & 31u;
          uint64_t xd = 0;
          if (sl < nd) xd = sl == dc ? (w ? w[0] : L.commit_time[p]) : (w ? w[2 + sl] : L.snap_vc[(uint64_t)sl * stride + p]);
          const bool failx = sl < nd && (!((u.spres >> sl) & 1u) || xd > vS);
          const bool included = row_or_u32(failx ? 1u : 0u) == 0;
          if (sl == 0) fl |= miss;
          if (!included) {
            mex = min(mex, q);
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
          for (uint32_t tt = 0; tt < NST; ++tt)
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
      for (uint32_t t = 0; t < NST; ++t) {
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
      const uint32_t count = cnt + ecnt;
      const uint32_t flags = row_or_u32(fl);
      const uint32_t minq = mex;
      uint64_t myct = (dl && cnt) ? in.K + mxl : 0;  // lane d: LastOpCt entry d
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

template <int D, bool LAG>
int launch_dl(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S, am_retry next) {
  static int occ = 0;
  if (!occ && (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_bc_rows<D, LAG>, BLOCK, 0) != hipSuccess || occ < 1))
    occ = 1;
  const uint64_t batches = (B->n_reads + WAVE - 1) / WAVE;
  uint64_t blocks = (batches + BLOCK / WAVE - 1) / (BLOCK / WAVE), cap = (uint64_t)ctx->n_cu * occ;
  if (blocks > cap) blocks = cap;
  if (blocks == 0) return AM_OK;
  hipLaunchKernelGGL((k_bc_rows<D, LAG>), dim3((unsigned)blocks), dim3(BLOCK), 0, ctx->stream, *L, *B, *R, S, next);
  AM_HIP(hipGetLastError());
  return AM_OK;
}

// the lag view at D > 8 where the store has one (#ifndef AM_BCR_LAG: on)
#ifndef AM_BCR_LAG
#define AM_BCR_LAG 1
#endif
template <int D>
int launch_d(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S, am_retry next) {
  if constexpr (D > 8 && AM_BCR_LAG)
    if (L->lag_ct && L->lag && L->key_lag) return launch_dl<D, true>(ctx, L, B, R, S, next);
  return launch_dl<D, false>(ctx, L, B, R, S, next);
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
