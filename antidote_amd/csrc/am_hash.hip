// am_hash.hip -- materialize/4 for add-wins-set / MV-register reads of moderate length
// (the tier between the 16-lane row tier, am_rows.hip, and the LDS-sort tier,
// am_sets.hip), over the packed streaming view and the set-effect record view.
//
// The closed form of am_sets.hip: a birth (a, tok) at position p survives iff no kill
// of the same kill key (AW: (tok, elem); MV: tok) sits at q > p.  Per kill key that
// is the same as
//     survives  <=>  max birth position >= max kill position
// (a kill at the birth's own position does not kill it: same-op add wins, MV removes
// before inserting; base-snapshot pairs are births at -1).  So no sort is needed.  Two
// kernels:
//   k_stream (set mode, am_stream.h)  the HBM-bound part: the reads' ops stream through
//       the wave-per-64-reads pipeline of the PN/LWW kernel (packed view, double-buffered
//       256-op tiles); is_op_in_snapshot/7 per op; it writes every scalar output of
//       materialize/4 and, per read, an included-op bitmap and a task (read, record range);
//   k_hrec  one workgroup per read: the read's records (a, tok, op|kill) of included ops
//       go into an LDS open-addressing table keyed by the token (64-bit LDS CAS, linear
//       probing) holding `a` (AW elem / MV value) and two LDS atomicMax positions; the
//       slots with max birth >= max kill are the survivors, compacted, rank-sorted by
//       (a, tok) (distinct keys) and written as CSR.
// Exactness guards (each hands the read to the LDS-sort tier, which redoes it from
// scratch, so every read is still materialized bit-exactly): a token with two different
// `a` (AW: one token under two elems; MV: two values), the sentinel in a token or `a`,
// more than MAXPROBE probes, more survivors than SCAP, logs longer than HOPS ops.
#include "am_block.h"
#include "am_stream.h"  // am_setincl, HB_WORDS

using namespace amk;
using amk_stream::HB_WORDS;

namespace {

constexpr int BLOCK = 256;
constexpr int RPT = 6;                               // records per thread per pass
constexpr uint64_t RPASS = (uint64_t)BLOCK * RPT;
constexpr uint32_t HOPS = 2048;                      // longest log of the tier (bitmap: HB_WORDS words)
static_assert((HOPS + 3 + 255) / 256 * 8 <= HB_WORDS, "bitmap slot too small");
constexpr uint64_t TEMPTY = ~0ull;
constexpr int32_t PNONE = (int32_t)0x80000000;
constexpr uint32_t MAXPROBE = 64;

template <int HCAP>
struct HSmem {
  static constexpr uint32_t SCAP = HCAP / 2;
  uint64_t tok[HCAP];            // slot key (TEMPTY: free)
  uint64_t a[HCAP];              // AW elem / MV value of the token (TEMPTY: not yet known)
  int32_t mb[HCAP], mk[HCAP];    // max birth / kill position (PNONE: none)
  uint32_t incl[HB_WORDS];       // included ops of the read (bit = position in the key + (off0 & 3))
  uint64_t surv[2 * SCAP];       // survivors as (a, tok) pairs (16-byte LDS loads)
  uint32_t ctr[4];               // [0] survivors [1] guard tripped
};

template <int HCAP>
__device__ __forceinline__ uint32_t slot_of(uint64_t tok) {
  constexpr int BITS = __builtin_ctz(HCAP);
  return (uint32_t)((tok * 0x9E3779B97F4A7C15ull) >> (64 - BITS));
}

// one birth / kill of token `tok` with `a` at `pos` (check_a: `a` is part of the key)
template <int HCAP>
__device__ __forceinline__ void put(HSmem<HCAP> &s, uint64_t a, uint64_t tok, int32_t pos, bool kill, bool check_a) {
  if (tok == TEMPTY || (check_a && a == TEMPTY)) {
    s.ctr[1] = 1;
    return;
  }
  uint32_t h = slot_of<HCAP>(tok);
  uint32_t probe = 0;
  for (;; ++probe) {
    if (probe == MAXPROBE) {
      s.ctr[1] = 1;
      return;
    }
    const uint64_t old = atomicCAS((unsigned long long *)&s.tok[h], (unsigned long long)TEMPTY, (unsigned long long)tok);
    if (old == TEMPTY || old == tok) break;
    h = (h + 1) & (HCAP - 1);
  }
  if (check_a) {
    const uint64_t olda = atomicCAS((unsigned long long *)&s.a[h], (unsigned long long)TEMPTY, (unsigned long long)a);
    if (olda != TEMPTY && olda != a) s.ctr[1] = 1;
  }
  atomicMax(kill ? &s.mk[h] : &s.mb[h], pos);
}


// one read's first record pass (RPT records per thread) + its bitmap word, in registers
struct RecBuf {
  uint64_t a[RPT], b[RPT];
  uint32_t m[RPT];
  uint32_t bm;
};
struct Task {
  uint64_t tr, rk0, rk1;
};

// Reads are software-pipelined: while read i is resolved, the records and bitmap of read
// i + G are in flight and the task of read i + 2G (G = grid size), so the HBM latency
// of the dependent chain task -> records overlaps the LDS work of the current read.
template <int TYPE, int HCAP>
__global__ void __launch_bounds__(BLOCK, 4) k_hrec(am_op_log L, am_read_batch B, am_read_result R, am_sel S,
                                                am_setincl X, am_retry next, uint32_t dbg) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  HSmem<HCAP> &s = *reinterpret_cast<HSmem<HCAP> *>(smem_raw);
  constexpr uint32_t SCAP = HSmem<HCAP>::SCAP;
  const uint32_t tid = threadIdx.x;
  const uint64_t nsel = S.idx ? (uint64_t)(uniform_u32(S.range[1]) - uniform_u32(S.range[0])) : B.n_reads;
  const uint64_t G = gridDim.x;

  auto load_task = [&](uint64_t i, Task &t) {
    t.tr = 1ull << 32, t.rk0 = 0, t.rk1 = 0;  // past the end: flag 1 (nothing to do)
    if (i < nsel) {
      t.tr = uniform_u64(X.task_r[i]);
      t.rk0 = uniform_u64(X.task_rk[2 * i]);
      t.rk1 = uniform_u64(X.task_rk[2 * i + 1]);
    }
  };
  auto load_recs = [&](uint64_t i, const Task &t, uint64_t q0, RecBuf &rb) {
    const bool live = ((t.tr >> 32) & 0xFFu) == 0;
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
      const uint64_t q = q0 + (uint64_t)j * BLOCK + tid;
      if (live && q < t.rk1) rb.a[j] = L.rec_a[q], rb.b[j] = L.rec_b[q], rb.m[j] = L.rec_meta[q];
      else rb.m[j] = 0xFFFFFFFFu;
    }
    rb.bm = (live && q0 == t.rk0 && tid < HB_WORDS) ? X.bitmap[i * HB_WORDS + tid] : 0u;
  };
  auto put_recs = [&](const RecBuf &rb, uint32_t sh) {
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
      const uint32_t m = rb.m[j];
      if (m == 0xFFFFFFFFu) continue;
      const uint32_t bit = AM_REC_OP(m) + sh;
      if (bit >= HB_WORDS * 32 || !((s.incl[bit >> 5] >> (bit & 31)) & 1u)) continue;
      const bool kill = (m & AM_REC_KILL) != 0;
      if (dbg & 1) {
        if ((rb.a[j] ^ rb.b[j]) == 0x1234567ull) s.ctr[2] = 1;
        continue;
      }
      put<HCAP>(s, rb.a[j], rb.b[j], (int32_t)AM_REC_OP(m), kill, TYPE == AM_AWSET || !kill);
    }
  };

  Task tc, tn, tf;
  RecBuf cur, nxt;
  uint64_t i = blockIdx.x;
  load_task(i, tc);
  load_task(i + G, tn);
  load_recs(i, tc, tc.rk0, cur);
  for (; i < nsel; i += G) {
    load_task(i + 2 * G, tf);
    load_recs(i + G, tn, tn.rk0, nxt);

    const uint32_t flag = (uint32_t)(tc.tr >> 32) & 0xFFu;
    const uint32_t r = (uint32_t)tc.tr, sh = (uint32_t)(tc.tr >> 40) & 3u;
    if (flag == 2) {  // longer than HOPS: the LDS-sort tier (or the big-read tier)
      if (tid == 0) next.list[atomicAdd(next.count, 1u)] = r;
    } else if (flag == 0) {  // flag 1: error status written by k_stream
      for (uint32_t k = tid; k < (uint32_t)HCAP && !(dbg & 4); k += BLOCK) {
        s.tok[k] = TEMPTY;
        s.a[k] = TEMPTY;
        s.mb[k] = PNONE;
        s.mk[k] = PNONE;
      }
      if (tid < HB_WORDS) s.incl[tid] = cur.bm;
      if (tid < 4) s.ctr[tid] = 0;
      __syncthreads();
      if (B.base.set_off) {  // base snapshot pairs: births at -1
        const uint64_t bo = B.base.set_off[r];
        const uint32_t bl = B.base.set_len[r];
        for (uint32_t k = tid; k < bl; k += BLOCK)
          put<HCAP>(s, B.base.set_a[bo + k], B.base.set_b[bo + k], -1, false, true);
      }
      // records of the included ops -> the token table (first pass prefetched)
      put_recs(cur, sh);
      for (uint64_t q0 = tc.rk0 + RPASS; q0 < tc.rk1; q0 += RPASS) {
        load_recs(i, tc, q0, cur);  // cur is consumed: reuse its registers
        put_recs(cur, sh);
      }
      __syncthreads();
      // survivors: compact, rank-sort by (a, tok), write the CSR
      for (uint32_t k = tid; k < (uint32_t)HCAP; k += BLOCK) {
        const int32_t b = s.mb[k];
        if (b != PNONE && b >= s.mk[k]) {
          const uint32_t o = atomicAdd(&s.ctr[0], 1u);
          if (o < SCAP) s.surv[2 * o] = s.a[k], s.surv[2 * o + 1] = s.tok[k];
        }
      }
      __syncthreads();
      const uint32_t ns = (dbg & 2) ? 0u : s.ctr[0];
      // pad to a multiple of 8 with (~0, ~0): above every real pair (a = ~0 trips the guard)
      const uint32_t ns8 = (ns + 7) & ~7u;
      if (ns <= SCAP && tid < ns8 - ns) s.surv[2 * (ns + tid)] = TEMPTY, s.surv[2 * (ns + tid) + 1] = TEMPTY;
      __syncthreads();
      if (s.ctr[1] || ns > SCAP) {  // exactness guard tripped: the LDS-sort tier redoes the read
        if (tid == 0) next.list[atomicAdd(next.count, 1u)] = r;
      } else {
        const uint64_t ooff = R.value.set_off[r], ocap = R.value.set_off[r + 1] - ooff;
        if (ns > ocap) {
          if (tid == 0) R.status[r] = AM_ERR_CAPACITY;
        } else {
          // rank = number of smaller pairs (keys are distinct); the LDS reads are wave
          // broadcasts, 8 in flight per step
          const u64x2 *sv = reinterpret_cast<const u64x2 *>(s.surv);
          for (uint32_t k = tid; k < ns; k += BLOCK) {
            const u64x2 me = sv[k];
            uint32_t rank = 0;
            for (uint32_t j = 0; j < ns8; j += 8) {
              u64x2 c[8];
#pragma unroll
              for (int q = 0; q < 8; ++q) c[q] = sv[j + q];
#pragma unroll
              for (int q = 0; q < 8; ++q) rank += (c[q].x < me.x || (c[q].x == me.x && c[q].y < me.y)) ? 1u : 0u;
            }
            R.value.set_a[ooff + rank] = me.x;
            R.value.set_b[ooff + rank] = me.y;
          }
          if (tid == 0) R.value.set_len[r] = ns;
        }
      }
      __syncthreads();
    }
    tc = tn;
    tn = tf;
    cur = nxt;
  }
}

template <int TYPE>
int launch_t(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S, am_retry next) {
  constexpr int HCAP = 1024;
  const uint64_t n = B->n_reads;
  // scratch: task_r [n] u64, task_rk [2n] u64, bitmap [n][HB_WORDS] u32
  void *scr = nullptr;
  int rc = am_ctx_scratch(ctx, AM_SCR_HASHX, n * (3 * sizeof(uint64_t) + HB_WORDS * sizeof(uint32_t)) + 64, &scr);
  if (rc) return rc;
  am_setincl X;
  X.task_r = (uint64_t *)scr;
  X.task_rk = X.task_r + n;
  X.bitmap = (uint32_t *)(X.task_rk + 2 * n);
  X.max_ops = HOPS;
  rc = am_launch_stream_sets(ctx, L, B, R, S, TYPE, X);
  if (rc) return rc;
  constexpr size_t smem = sizeof(HSmem<HCAP>);
  const char *dv = getenv("AM_HASH_DBG");  // A/B knob: 1 skip table inserts, 2 skip the sort, 4 skip the reset
  const uint32_t dbg = dv ? (uint32_t)strtoul(dv, nullptr, 10) : 0u;
  static int nb = 0;
  if (!nb) {
    AM_HIP(hipFuncSetAttribute((const void *)k_hrec<TYPE, HCAP>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_hrec<TYPE, HCAP>, BLOCK, smem) != hipSuccess || nb < 1)
      nb = 1;
  }
  uint64_t blocks = n, cap = (uint64_t)ctx->n_cu * (uint64_t)nb;
  if (blocks > cap) blocks = cap;
  if (blocks == 0) return AM_OK;
  hipLaunchKernelGGL((k_hrec<TYPE, HCAP>), dim3((unsigned)blocks), dim3(BLOCK), smem, ctx->stream, *L, *B, *R, S, X, next, dbg);
  AM_HIP(hipGetLastError());
  return AM_OK;
}

}  // namespace

bool am_hash_applies(const am_op_log *L, const am_read_result *R, uint32_t type) {
  const char *e = getenv("AM_HASH");
  if (e && e[0] == '0') return false;
  return (type == AM_AWSET || type == AM_MVREG) && am_log_packed(L) && L->rec_key_off && R->value.set_off &&
         R->value.set_len && R->value.set_a && R->value.set_b;
}

int am_launch_hash(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S,
                   uint32_t type, am_retry next) {
  switch (type) {
    case AM_AWSET: return launch_t<AM_AWSET>(ctx, L, B, R, S, next);
    case AM_MVREG: return launch_t<AM_MVREG>(ctx, L, B, R, S, next);
    default: return AM_ERR_UNSUPPORTED;
  }
}
