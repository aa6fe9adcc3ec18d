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
#include "am_stream.h"

using namespace amk;
using amk_stream::HB_WORDS;

namespace {

constexpr int BLOCK = 256;
constexpr int RPT = 8;                               // records per thread per pass
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
  uint64_t oa[SCAP], ob[SCAP];   // survivors
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


template <int TYPE, int HCAP>
__global__ void __launch_bounds__(BLOCK) k_hrec(am_op_log L, am_read_batch B, am_read_result R, am_sel S,
                                                am_setincl X, am_retry next) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  HSmem<HCAP> &s = *reinterpret_cast<HSmem<HCAP> *>(smem_raw);
  constexpr uint32_t SCAP = HSmem<HCAP>::SCAP;
  const uint32_t tid = threadIdx.x;
  const uint64_t nsel = S.idx ? (uint64_t)(uniform_u32(S.range[1]) - uniform_u32(S.range[0])) : B.n_reads;
  for (uint64_t i = blockIdx.x; i < nsel; i += gridDim.x) {
    const uint64_t tr = uniform_u64(X.task_r[i]);
    const uint32_t flag = (uint32_t)(tr >> 32) & 0xFFu;
    const uint32_t r = (uint32_t)tr, sh = (uint32_t)(tr >> 40) & 3u;
    if (flag == 1) continue;  // error status written by k_stream
    if (flag == 2) {          // longer than HOPS: the LDS-sort tier (or the big-read tier)
      if (tid == 0) next.list[atomicAdd(next.count, 1u)] = r;
      continue;
    }
    const uint64_t rk0 = uniform_u64(X.task_rk[2 * i]), rk1 = uniform_u64(X.task_rk[2 * i + 1]);
    for (uint32_t k = tid; k < (uint32_t)HCAP; k += BLOCK) {
      s.tok[k] = TEMPTY;
      s.a[k] = TEMPTY;
      s.mb[k] = PNONE;
      s.mk[k] = PNONE;
    }
    if (tid < HB_WORDS) s.incl[tid] = X.bitmap[i * HB_WORDS + tid];
    if (tid < 4) s.ctr[tid] = 0;
    __syncthreads();
    if (B.base.set_off) {  // base snapshot pairs: births at -1
      const uint64_t bo = B.base.set_off[r];
      const uint32_t bl = B.base.set_len[r];
      for (uint32_t k = tid; k < bl; k += BLOCK) put<HCAP>(s, B.base.set_a[bo + k], B.base.set_b[bo + k], -1, false, true);
    }
    // records of the included ops -> the token table
    for (uint64_t q0 = rk0; q0 < rk1; q0 += RPASS) {
      uint64_t ra[RPT], rb[RPT];
      uint32_t rm[RPT];
#pragma unroll
      for (int j = 0; j < RPT; ++j) {
        const uint64_t q = q0 + (uint64_t)j * BLOCK + tid;
        if (q < rk1) ra[j] = L.rec_a[q], rb[j] = L.rec_b[q], rm[j] = L.rec_meta[q];
        else rm[j] = 0xFFFFFFFFu;
      }
#pragma unroll
      for (int j = 0; j < RPT; ++j) {
        const uint32_t m = rm[j];
        if (m == 0xFFFFFFFFu) continue;
        const uint32_t bit = AM_REC_OP(m) + sh;
        if (bit >= HB_WORDS * 32 || !((s.incl[bit >> 5] >> (bit & 31)) & 1u)) continue;
        const bool kill = (m & AM_REC_KILL) != 0;
        put<HCAP>(s, ra[j], rb[j], (int32_t)AM_REC_OP(m), kill, TYPE == AM_AWSET || !kill);
      }
    }
    __syncthreads();
    // survivors: compact, rank-sort by (a, tok), write the CSR
    for (uint32_t k = tid; k < (uint32_t)HCAP; k += BLOCK) {
      const int32_t b = s.mb[k];
      if (b != PNONE && b >= s.mk[k]) {
        const uint32_t o = atomicAdd(&s.ctr[0], 1u);
        if (o < SCAP) s.oa[o] = s.a[k], s.ob[o] = s.tok[k];
      }
    }
    __syncthreads();
    const uint32_t ns = s.ctr[0];
    if (s.ctr[1] || ns > SCAP) {  // exactness guard tripped: the LDS-sort tier redoes the read
      if (tid == 0) next.list[atomicAdd(next.count, 1u)] = r;
      __syncthreads();
      continue;
    }
    const uint64_t ooff = R.value.set_off[r], ocap = R.value.set_off[r + 1] - ooff;
    if (ns > ocap) {
      if (tid == 0) R.status[r] = AM_ERR_CAPACITY;
    } else {
      for (uint32_t k = tid; k < ns; k += BLOCK) {
        const uint64_t ka = s.oa[k], kb = s.ob[k];
        uint32_t rank = 0;
        for (uint32_t j = 0; j < ns; ++j) {
          const uint64_t ja = s.oa[j], jb = s.ob[j];
          rank += (ja < ka || (ja == ka && jb < kb)) ? 1u : 0u;
        }
        R.value.set_a[ooff + rank] = ka;
        R.value.set_b[ooff + rank] = kb;
      }
      if (tid == 0) R.value.set_len[r] = ns;
    }
    __syncthreads();
  }
}

template <int D, int TYPE, bool GENERAL>
int launch_incl(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S,
                const am_setincl &X) {
  using namespace amk_stream;
  static int occ = 0;
  if (occ == 0) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_stream<D, TYPE, GENERAL, true>, amk_stream::BLOCK, 0) !=
            hipSuccess ||
        nb <= 0)
      nb = 2;
    occ = nb;
  }
  const uint64_t batches = (B->n_reads + WAVE - 1) / WAVE;
  uint64_t blocks = (batches + WPB - 1) / WPB;
  const uint64_t cap = (uint64_t)ctx->n_cu * (uint64_t)occ;
  if (blocks > cap) blocks = cap;
  if (blocks == 0) return AM_OK;
  hipLaunchKernelGGL((k_stream<D, TYPE, GENERAL, true>), dim3((unsigned)blocks), dim3(amk_stream::BLOCK), 0, ctx->stream,
                     *L, *B, *R, S, am_rows_cfg{}, X);
  AM_HIP(hipGetLastError());
  return AM_OK;
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
  const bool general = am_batch_general(L, B);
  const uint32_t nd = L->n_dc;
#define AM_I(D) rc = general ? launch_incl<D, TYPE, true>(ctx, L, B, R, S, X) : launch_incl<D, TYPE, false>(ctx, L, B, R, S, X);
  if (nd <= 1) AM_I(1)
  else if (nd <= 2) AM_I(2)
  else if (nd <= 3) AM_I(3)
  else if (nd <= 4) AM_I(4)
  else if (nd <= 8) AM_I(8)
  else if (nd <= 16) AM_I(16)
  else AM_I(32)
#undef AM_I
  if (rc) return rc;
  constexpr size_t smem = sizeof(HSmem<HCAP>);
  static int nb = 0;
  if (!nb) {
    AM_HIP(hipFuncSetAttribute((const void *)k_hrec<TYPE, HCAP>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_hrec<TYPE, HCAP>, BLOCK, smem) != hipSuccess || nb < 1)
      nb = 1;
  }
  uint64_t blocks = n, cap = (uint64_t)ctx->n_cu * (uint64_t)nb;
  if (blocks > cap) blocks = cap;
  if (blocks == 0) return AM_OK;
  hipLaunchKernelGGL((k_hrec<TYPE, HCAP>), dim3((unsigned)blocks), dim3(BLOCK), smem, ctx->stream, *L, *B, *R, S, X, next);
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
