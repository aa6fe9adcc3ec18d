// am_bcwave.hip -- materialize/4 for bounded-counter reads between the row tier and the
// big-read tier: one WAVE per read (antidote_crdt_counter_b: orddict:update_counter on
// P[{From,To}] and D[Id] is a keyed sum, folded by clocksi_materializer:apply_operations/4,
// src/clocksi_materializer.erl:113-121).
//
// The LDS-sort tier (am_sets.hip) gives such a read a 256-thread workgroup and 78 KB of LDS
// sized for set births/kills, so a CU holds two reads and most of a workgroup idles on a
// few hundred ops.  A counter read needs only its D*D + D slot sums: here each wave of a
// 256-thread block owns one read at a time with 20 B of LDS per slot (5.4 KB at D = 16):
//   * slots start at the base value (bc_base: row r of the base arrays, or a snapshot-cache
//     entry in the value pool);
//   * the read's ops stream in 256-op tiles over the packed view (am_wave.h incl4; escaped
//     ops from the full columns), payload words loaded with them (16-byte loads);
//   * every included amount goes into its slot with an exact 128-bit LDS accumulation
//     (64-bit atomics + carry, am_block.h acc128_atomic) and sets the slot's presence;
//   * scalar outputs come from wave reductions, the slots leave with coalesced stores and an
//     int64 overflow check (AM_ERR_OVERFLOW where Erlang would return a bignum).
// Reads it does not take (longer than BCW_OPS, n_dc > 16, no packed view) go to `next`.
#include "am_block.h"

using namespace amk;

namespace {

constexpr int BLOCK = 256;
constexpr int NW = BLOCK / WAVE;
constexpr int OPL = 4;
constexpr uint64_t BCW_OPS = AM_BCWAVE_OPS;  // longer logs: the chunked big-read tier

template <int DMAX>
struct BcSmem {
  static constexpr uint32_t NS = DMAX * DMAX + DMAX;
  uint64_t lo[NS];
  int64_t hi[NS];
  uint32_t pres[NS];
  uint64_t emx[DMAX];  // batch-clock kernel: LastOpCt maxima of the included escaped ops
};

// per-read inputs, wave-uniform (every lane reads the same read; GENERAL false: the batch clock)
template <int DMAX, bool GENERAL>
__device__ __forceinline__ void bc_inputs(const am_op_log &L, const am_read_batch &B, uint32_t nd, uint64_t r,
                                          ReadU<DMAX> &u) {
  const uint64_t n = B.n_reads;
  u.allmask = nd >= 32 ? 0xFFFFFFFFu : ((1u << nd) - 1u);
  const uint64_t rstride = (GENERAL && B.per_read_clock) ? n : 1, ridx = (GENERAL && B.per_read_clock) ? r : 0;
  u.spres = uniform_u32(B.read_pres[ridx]) & u.allmask;
  u.base_ignore = !GENERAL || !B.base_ignore || B.base_ignore[r];
  u.cpres = u.base_ignore ? 0u : (uniform_u32(B.base_pres[r]) & u.allmask);
#pragma unroll
  for (int d = 0; d < DMAX; ++d) {
    u.S[d] = (d < (int)nd && ((u.spres >> d) & 1u)) ? uniform_u64(B.read_vc[(uint64_t)d * rstride + ridx]) : 0;
    u.C0[d] = (d < (int)nd && ((u.cpres >> d) & 1u)) ? uniform_u64(B.base_vc[(uint64_t)d * n + r]) : 0;
  }
  u.has_txid = GENERAL && B.txid && (!B.txid_valid || B.txid_valid[r]) && L.op_txid;
  u.txid = u.has_txid ? uniform_u64(B.txid[r]) : 0;
}

// GENERAL false (the batch clock, no bases / TxIds / op presence): the clock is read once per
// wave and the tile loop tests the packed entries only; escaped ops (outside the packed view)
// are evaluated from the full columns in a pass of their own after the loop, so the loop holds
// neither the base thresholds nor the full-width accumulators (C5: 252 -> fewer VGPRs).
template <int DMAX, bool GENERAL>
__global__ void __launch_bounds__(BLOCK) k_bc_wave(am_op_log L, am_read_batch B, am_read_result R, am_sel S,
                                                   am_retry next) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  BcSmem<DMAX> &s = reinterpret_cast<BcSmem<DMAX> *>(smem_raw)[threadIdx.x >> 6];
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  const uint32_t nd = L.n_dc, np = nd * nd, ns = np + nd;
  const uint64_t n = B.n_reads;
  const uint64_t stride = L.snap_stride ? L.snap_stride : L.n_ops;
  const uint32_t sel0 = S.idx ? uniform_u32(S.range[0]) : 0u;
  const uint64_t nsel = S.idx ? (uint64_t)(uniform_u32(S.range[1]) - sel0) : n;
  const uint64_t W = (uint64_t)gridDim.x * NW;
  ReadU<DMAX> u;
  if (!GENERAL) bc_inputs<DMAX, false>(L, B, nd, 0, u);
  for (uint64_t i = (uint64_t)blockIdx.x * NW + uniform_u32(threadIdx.x >> 6); i < nsel; i += W) {
    const uint64_t r = S.idx ? (uint64_t)uniform_u32(S.idx[sel0 + i]) : i;
    const uint64_t key = uniform_u64(B.key[r]);
    const uint32_t rtype = uniform_u32(B.type[r]);
    int32_t status = AM_OK;
    uint64_t off0 = 0, off1 = 0;
    if (key >= L.n_keys) {
      status = AM_ERR_INVALID;
    } else {
      off0 = uniform_u64(L.key_off[key]);
      off1 = uniform_u64(am_kend(L, key));
      const uint32_t ktype = uniform_u32(L.key_type[key]);
      const uint32_t kfl = L.key_flags ? uniform_u32(L.key_flags[key]) : 0u;
      if (off1 > off0 && (ktype != rtype || (kfl & AM_KEY_MIXED_TYPES))) status = AM_ERR_CORRUPTED_OPS_CACHE;
      else if (rtype != (uint32_t)AM_BCOUNTER) status = AM_ERR_INVALID;
    }
    if (status != AM_OK) {
      if (lane == 0) R.status[r] = status, R.flags[r] = 0;
      continue;
    }
    if (off1 - off0 > BCW_OPS) {
      if (lane == 0) next.list[atomicAdd(next.count, 1u)] = (uint32_t)r;
      continue;
    }
    if (GENERAL) bc_inputs<DMAX, true>(L, B, nd, r, u);
    PkRead<DMAX> pk;
    pk_setup(u, nd, uniform_u64(L.key_tbase[key]), pk);
    LagRead<DMAX> lr;  // the batch clock at D > 8 reads the lag view where the store has one
    lag_setup(L, nd, key, !GENERAL && DMAX > 8 && L.lag_ct != nullptr, lr);
    // slots start at the base value (orddict entries present in the base stay present)
    if (lane < DMAX) s.emx[lane] = 0;
    for (uint32_t k = lane; k < ns; k += WAVE) {
      uint32_t bp = 0;
      const int64_t bv = GENERAL ? bc_base(B, r, np, nd, k, bp) : 0;
      s.lo[k] = (uint64_t)bv;
      s.hi[k] = bv < 0 ? -1 : 0;
      s.pres[k] = bp;
    }
    wave_sync();

    Acc<DMAX> a;  // GENERAL false: only after the tile loop (escaped ops, the fold)
    AccP<DMAX> ap;
    if (GENERAL) a.reset();
    ap.reset();
    // an included op's amount into its slot (exact 128-bit LDS sum) and the slot's presence
    auto apply = [&](uint32_t meta, int64_t v, uint64_t ft) {
      if (meta & AM_META_BAD) return;  // reported through FLAG_BAD
      const uint32_t kind = AM_META_KIND(meta);
      const uint32_t from = (uint32_t)(ft & 0xFF), to = (uint32_t)((ft >> 8) & 0xFF);
      if (kind > AM_BC_TRANSFER || from >= nd || to >= nd) {  // Type:update/2 would raise
        a.flags |= FLAG_BAD;
        return;
      }
      const uint32_t slot = kind == AM_BC_DECREMENT ? np + from : from * nd + (kind == AM_BC_INCREMENT ? from : to);
      acc128_atomic(&s.lo[slot], &s.hi[slot], v < 0 ? -1 : 0, (uint64_t)v);
      atomicOr(&s.pres[slot], 1u);
    };
    bool esc = false;
    // ops per lane: 4 (16-byte loads); the batch-clock kernel at D > 8 takes 2 so the loaded
    // entries (OL x D) leave room for a third wave per SIMD
    constexpr int OL = (!GENERAL && DMAX > 8) ? 2 : OPL;
    constexpr uint64_t TL = (uint64_t)WAVE * OL;
    for (uint64_t t = off0 & ~(uint64_t)(OL - 1); t < off1; t += TL) {
      const uint64_t g = t + (uint64_t)lane * OL;
      if (g >= off1) continue;
      uint32_t meta4;
      uint64_t amt[OL], ft[OL];
      if constexpr (OL == 4) {
        meta4 = *(const uint32_t *)(L.op_meta + g);
        const u64x2 a01 = *(const u64x2 *)(L.p0 + g), a23 = *(const u64x2 *)(L.p0 + g + 2);
        const u64x2 f01 = *(const u64x2 *)(L.p1 + g), f23 = *(const u64x2 *)(L.p1 + g + 2);
        amt[0] = a01.x, amt[1] = a01.y, amt[2] = a23.x, amt[3] = a23.y;
        ft[0] = f01.x, ft[1] = f01.y, ft[2] = f23.x, ft[3] = f23.y;
      } else {
        meta4 = *(const uint16_t *)(L.op_meta + g);
        const u64x2 a01 = *(const u64x2 *)(L.p0 + g), f01 = *(const u64x2 *)(L.p1 + g);
        amt[0] = a01.x, amt[1] = a01.y, ft[0] = f01.x, ft[1] = f01.y;
      }
      uint32_t ib;
      if constexpr (GENERAL) {
        ib = incl4<DMAX, true>(L, nd, stride, u, pk, g, off0, off1, ap, a);
      } else if (DMAX > 8 && lr.on) {  // 4 + 2 D bytes per op
        static_assert(GENERAL || DMAX <= 8 || OL == 2, "the lag loads below take 2 ops per lane");
        typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
        const u32x2_t cv = *(const u32x2_t *)(L.lag_ct + g);
        const uint32_t c[OL] = {cv.x, cv.y};
        uint32_t lw[DMAX][(OL + 1) / 2];
        uint64_t tx[OL] = {};
#pragma unroll
        for (int d = 0; d < DMAX; ++d) lw[d][0] = d < (int)nd ? *(const uint32_t *)(L.lag + (uint64_t)d * stride + g) : 0u;
        ib = pk_tile_lag<DMAX, OL, false>(u, pk, lr, c, lw, tx, g, off0, off1, ap, esc);
      } else {
        uint32_t x[OL][DMAX];
        uint64_t tx[OL];
#pragma unroll
        for (int k = 0; k < OL; ++k) tx[k] = 0;
#pragma unroll
        for (int d = 0; d < DMAX; ++d) {
          uint32_t q[OL];
          if constexpr (OL == 4) {
            u32x4 v = {0, 0, 0, 0};
            if (d < (int)nd) v = *(const u32x4 *)(L.pk_vc + (uint64_t)d * stride + g);
            q[0] = v.x, q[1] = v.y, q[2] = v.z, q[3] = v.w;
          } else {
            typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
            u32x2_t v = {0, 0};
            if (d < (int)nd) v = *(const u32x2_t *)(L.pk_vc + (uint64_t)d * stride + g);
            q[0] = v.x, q[1] = v.y;
          }
#pragma unroll
          for (int k = 0; k < OL; ++k) x[k][d] = q[k];
        }
        ib = pk_tile<DMAX, OL, false>(u, pk, x, tx, g, off0, off1, ap, esc);
      }
#pragma unroll
      for (int k = 0; k < OL; ++k)
        if ((ib >> k) & 1u) apply((meta4 >> (8 * k)) & 0xFFu, (int64_t)amt[k], ft[k]);
    }
    if (!GENERAL) a.reset();
    if constexpr (!GENERAL && DMAX <= 8) {
      if (__ballot(esc)) {  // rare: ops outside the packed view, from the full columns
        for (uint64_t p = off0 + lane; p < off1; p += WAVE) {
          if (L.pk_vc[p] != AM_PK_ESC) continue;
          uint64_t sv[DMAX], ct;
          uint32_t meta;
          esc_load<DMAX>(L, nd, stride, p, sv, ct, meta);
          if (eval_op<DMAX, false>(u, meta, ct, sv, u.allmask, false, p, a))
            apply(meta, (int64_t)L.p0[p], L.p1[p]);
        }
      }
    } else if constexpr (!GENERAL) {
      if (__ballot(esc)) {
        // D > 8: the same, eval_op<DMAX, false> one DC at a time (the clock entry from lane d)
        // and the included ops' maxima into LDS, so the pass holds no D-wide arrays (it would
        // set the kernel's register peak)
        uint64_t vS = 0;
#pragma unroll
        for (int d = 0; d < DMAX; ++d) vS = (uint32_t)d == lane ? u.S[d] : vS;
        const uint32_t *escv = lr.on ? L.lag_ct : L.pk_vc;  // the view the loop streamed
        for (uint64_t p = off0 + lane; p < off1; p += WAVE) {
          if (escv[p] != AM_PK_ESC) continue;
          const uint64_t *w = esc_row(L, stride, p);  // its escape row, or the columns
          const uint32_t meta = w ? (uint32_t)w[1] : L.op_meta[p], dc = meta & 31u;
          const uint64_t ct = w ? w[0] : L.commit_time[p];
          bool incl = true;
          for (uint32_t d = 0; d < nd; ++d) {
            if (!((u.spres >> d) & 1u)) {  // logger:error("Could not find DC in SS"); excluded
              incl = false;
              a.flags |= AM_FLAG_MISSING_DC_LOGGED;
              continue;
            }
            const uint64_t x = d == dc ? ct : (w ? w[2 + d] : L.snap_vc[(uint64_t)d * stride + p]);
            incl &= x <= lane_u64(vS, d);
          }
          if (!incl) {
            a.min_excl = p < a.min_excl ? p : a.min_excl;
            continue;
          }
          for (uint32_t d = 0; d < nd; ++d) {
            const uint64_t x = d == dc ? ct : (w ? w[2 + d] : L.snap_vc[(uint64_t)d * stride + p]);
            atomicMax((unsigned long long *)&s.emx[d], (unsigned long long)x);
          }
          a.pres |= u.allmask;
          a.count += 1;
          if (meta & AM_META_BAD) a.flags |= FLAG_BAD;
          apply(meta, (int64_t)L.p0[p], L.p1[p]);
        }
        wave_sync();
#pragma unroll
        for (int d = 0; d < DMAX; ++d) a.mx[d] = d < (int)nd ? s.emx[d] : 0;
      }
    }
    pk_fold(ap, pk.K, u.allmask, a);
    wave_sync();

    // ---- scalar outputs (wave reductions, results in every lane) ----
    const uint32_t count = wave_sum_u32_v(a.count), flags = wave_or_u32_v(a.flags), pres = wave_or_u32_v(a.pres);
    const uint64_t min_excl = wave_min_u64_v(a.min_excl);
    uint64_t myct = 0;  // lane d: max X[d] over the included ops
#pragma unroll
    for (int d = 0; d < DMAX; ++d) {
      if (d >= (int)nd) continue;
      const uint64_t m = wave_max_u64_v(a.mx[d]);
      if ((uint32_t)d == lane) myct = m;
    }
    status = (flags & FLAG_BAD) ? AM_ERR_UNEXPECTED_OPERATION : AM_OK;
    // the slots' LDS words read once, all up front (lane l: slots l, l + 64, ...)
    constexpr uint32_t NC = (BcSmem<DMAX>::NS + WAVE - 1) / WAVE;
    uint64_t slo[NC];
    uint32_t spr[NC];
    bool ovf = false;
#pragma unroll
    for (uint32_t c = 0; c < NC; ++c) {
      const uint32_t k = c * WAVE + lane;
      slo[c] = k < ns ? s.lo[k] : 0ull;
      spr[c] = k < ns ? s.pres[k] : 0u;
      ovf |= k < ns && s.hi[k] != ((int64_t)slo[c] < 0 ? -1 : 0);
    }
    if (status == AM_OK && __ballot(ovf)) status = AM_ERR_OVERFLOW;
    uint32_t nent = 0;
    if (status == AM_OK) {  // the present slots as (slot, value) pairs, slot order
      const uint64_t so = R.value.set_off[r], cap = R.value.set_off[r + 1] - so;
#pragma unroll
      for (uint32_t c = 0; c < NC; ++c) {
        const uint32_t k = c * WAVE + lane;
        const bool p = k < ns && spr[c] != 0;
        const uint64_t m = __ballot(p);
        const uint64_t pos = nent + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        if (p && pos < cap) R.value.set_a[so + pos] = k, R.value.set_b[so + pos] = slo[c];
        nent += (uint32_t)__popcll(m);
      }
      if (nent > cap) status = AM_ERR_CAPACITY;
    }
    const bool ign = u.base_ignore && count == 0;
    const uint32_t opres = ign ? 0u : (pres | u.cpres);
    if (status == AM_OK && lane < nd) {
      uint64_t c0 = 0;
#pragma unroll
      for (int d = 0; d < DMAX; ++d)
        if ((uint32_t)d == lane) c0 = u.C0[d];
      R.last_ct[(uint64_t)lane * n + r] = ((opres >> lane) & 1u) ? (myct > c0 ? myct : c0) : 0;
    }
    if (lane == 0) {
      R.status[r] = status;
      R.flags[r] = (uint8_t)(flags & 0xFFu);
      if (status == AM_OK) {
        const uint64_t idb = L.key_id_base ? L.key_id_base[key] : 1;
        const uint64_t nops = off1 - off0;
        int64_t nlo;
        if (min_excl != NONE)
          nlo = (L.op_id ? (int64_t)L.op_id[min_excl] : (int64_t)(idb + (min_excl - off0))) - 1;
        else
          nlo = nops == 0 ? 0 : (L.op_id ? (int64_t)L.op_id[off1 - 1] : (int64_t)(idb + nops - 1));
        R.new_last_op[r] = nlo;
        R.last_ct_ignore[r] = ign ? 1 : 0;
        R.last_ct_pres[r] = opres;
        R.is_new_ss[r] = count > 0;
        R.count[r] = count;
        R.value.set_len[r] = nent;
      }
    }
    wave_sync();  // the slots are rewritten by the wave's next read
  }
}

template <int D, bool GENERAL>
int launch_dg(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S, am_retry next) {
  constexpr size_t smem = sizeof(BcSmem<D>) * NW;
  static int occ = 0;
  if (!occ) {
    AM_HIP(hipFuncSetAttribute((const void *)k_bc_wave<D, GENERAL>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)smem));
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_bc_wave<D, GENERAL>, BLOCK, smem) != hipSuccess || occ < 1)
      occ = 1;
  }
  uint64_t blocks = (B->n_reads + NW - 1) / NW, cap = (uint64_t)ctx->n_cu * occ;
  if (blocks > cap) blocks = cap;
  if (blocks == 0) return AM_OK;
  hipLaunchKernelGGL((k_bc_wave<D, GENERAL>), dim3((unsigned)blocks), dim3(BLOCK), smem, ctx->stream, *L, *B, *R, S,
                     next);
  AM_HIP(hipGetLastError());
  return AM_OK;
}
template <int D>
int launch_d(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S, am_retry next) {
  return am_batch_general(L, B) ? launch_dg<D, true>(ctx, L, B, R, S, next) : launch_dg<D, false>(ctx, L, B, R, S, next);
}

}  // namespace

bool am_bcwave_applies(const am_op_log *L, const am_read_result *R) {
  return am_log_packed(L) && L->n_dc <= 16 && L->op_meta && R->value.set_off && R->value.set_len && R->value.set_a &&
         R->value.set_b;
}

int am_launch_bcwave(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S,
                     am_retry next) {
  const uint32_t nd = L->n_dc;
  if (nd <= 1) return launch_d<1>(ctx, L, B, R, S, next);
  if (nd <= 2) return launch_d<2>(ctx, L, B, R, S, next);
  if (nd <= 3) return launch_d<3>(ctx, L, B, R, S, next);
  if (nd <= 4) return launch_d<4>(ctx, L, B, R, S, next);
  if (nd <= 8) return launch_d<8>(ctx, L, B, R, S, next);
  return launch_d<16>(ctx, L, B, R, S, next);
}
