// am_materialize.hip -- batched clocksi_materializer:materialize/4 on gfx950.
//
// One wavefront (64 lanes) materializes one read = one key's op log.  Lanes
// stream the log in 256-op tiles: lane l owns ops [g, g+4) of the tile with
// g = tile + 4l, so every per-op column (op_meta u8, commit_time u64,
// snap_vc[d] u64, payload u64) is read with 4..32-byte-per-lane loads that
// coalesce into one contiguous 256..2048-byte segment per wave instruction.
//
// Per op the lane evaluates, branch-free across DCs (reference in brackets):
//   X = snapshot_time with X[commit_dc] := commit_time      [dict:store, clocksi_materializer.erl:224]
//   candidate = base ignore | !le(X, base_clock) | TxId match [belongs_to_snapshot_op, materializer.erl:102-106;
//                                                             is_op_in_snapshot :219-220]
//   included  = candidate & all_{d in X} (d in S & X[d] <= S[d])   [dict:fold, :236-258]
// and accumulates
//   * the union-max of included clocks (-> LastOpCt)          [dict:update, :249-256]
//   * the count and the type's commutative reduction of the included effects
//     (PN sum, LWW max over {Ts, Value}; bcounter keyed sums) [apply_operations :113-121]
//   * the position of the OLDEST excluded candidate (-> NewLastOp = its id - 1;
//     the newest->oldest walk of materialize_intern keeps overwriting FirstHole)
// then reduces across the wave with DPP/ds_swizzle shuffles.  The reference
// walks newest->oldest and folds oldest->newest; every quantity above is an
// associative, commutative reduction, so any lane order gives the same bits.
#include "am_internal.h"

namespace {

constexpr int WAVE = 64;
constexpr int BLOCK = 256;
constexpr int WPB = BLOCK / WAVE;
constexpr uint64_t NONE = ~0ull;
constexpr int OPL = 4;                 // ops per lane per tile
constexpr int TILE = WAVE * OPL;       // 256 ops per wave per tile

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    uint64_t w = __shfl_xor(v, o, WAVE);
    v = w > v ? w : v;
  }
  return v;
}
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    uint64_t w = __shfl_xor(v, o, WAVE);
    v = w < v ? w : v;
  }
  return v;
}
__device__ __forceinline__ uint32_t wave_or_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o, WAVE);
  return v;
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
  return v;
}
// exact 128-bit sum of per-lane (hi, lo) pairs
__device__ __forceinline__ void wave_sum_i128(int64_t &hi, uint64_t &lo) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    uint64_t wlo = __shfl_xor(lo, o, WAVE);
    int64_t whi = __shfl_xor(hi, o, WAVE);
    uint64_t s = lo + wlo;
    hi = hi + whi + (s < lo ? 1 : 0);
    lo = s;
  }
}

__device__ __forceinline__ uint32_t uniform_u32(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uniform_u64(uint64_t v) {
  uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}

template <int DMAX>
struct ReadU {        // wave-uniform inputs of one read
  uint64_t S[DMAX];   // MinSnapshotTime (absent lanes 0)
  uint64_t C0[DMAX];  // base snapshot_time (absent lanes 0)
  uint32_t spres, cpres, allmask;
  bool base_ignore, has_txid;
  uint64_t txid;
};

template <int DMAX>
struct Acc {
  uint64_t mx[DMAX];
  uint32_t pres = 0, count = 0, flags = 0;
  uint64_t min_excl = NONE;
};

#define FLAG_BAD 0x100u

// Evaluate one op; returns true when it is included in the snapshot.
template <int DMAX>
__device__ __forceinline__ bool eval_op(const ReadU<DMAX> &u, uint8_t meta, uint64_t ct, const uint64_t (&snap)[DMAX],
                                        uint32_t spres_op, bool txmatch, uint64_t pos, Acc<DMAX> &a) {
  const uint32_t dc = meta & 31u;
  const uint32_t xpres = (spres_op | (1u << dc)) & u.allmask;
  uint64_t X[DMAX];
#pragma unroll
  for (int d = 0; d < DMAX; ++d) X[d] = ((uint32_t)d == dc) ? ct : (((xpres >> d) & 1u) ? snap[d] : 0);
  bool cand = u.base_ignore | txmatch;
  if (!cand) {
    bool le = true;
#pragma unroll
    for (int d = 0; d < DMAX; ++d) le &= X[d] <= u.C0[d];
    cand = !le;
  }
  if (!cand) return false;
  bool incl = true;
#pragma unroll
  for (int d = 0; d < DMAX; ++d) {
    if ((xpres >> d) & 1u) {
      if ((u.spres >> d) & 1u) {
        incl &= X[d] <= u.S[d];
      } else {
        incl = false;
        a.flags |= AM_FLAG_MISSING_DC_LOGGED;
      }
    }
  }
  if (incl) {
#pragma unroll
    for (int d = 0; d < DMAX; ++d) a.mx[d] = X[d] > a.mx[d] ? X[d] : a.mx[d];
    a.pres |= xpres;
    a.count += 1;
    if (meta & AM_META_BAD) a.flags |= FLAG_BAD;
  } else {
    a.min_excl = pos < a.min_excl ? pos : a.min_excl;
  }
  return incl;
}

// ---- per-type value reductions ----
struct PnVal {
  int64_t hi = 0;
  uint64_t lo = 0;
  __device__ void add(uint64_t p0, uint64_t) {
    int64_t v = (int64_t)p0;
    uint64_t s = lo + (uint64_t)v;
    hi += (v < 0 ? -1 : 0) + (s < lo ? 1 : 0);
    lo = s;
  }
};
struct LwwVal {
  uint64_t ts = 0, val = 0;
  bool has = false;
  __device__ void add(uint64_t p0, uint64_t p1) {
    bool gt = !has || p0 > ts || (p0 == ts && p1 > val);
    ts = gt ? p0 : ts;
    val = gt ? p1 : val;
    has = true;
  }
};

template <int TYPE>
struct ValOf;
template <>
struct ValOf<AM_PN> {
  using T = PnVal;
  static constexpr bool NEED_P1 = false;
};
template <>
struct ValOf<AM_LWW> {
  using T = LwwVal;
  static constexpr bool NEED_P1 = true;
};

// Materialize read r (one wavefront).  TYPE is the read's (wave-uniform) type.
template <int DMAX, int TYPE>
__device__ __forceinline__ void read_scalar(const am_op_log &L, const am_read_batch &B, const am_read_result &R,
                                            uint64_t r, uint64_t key, uint64_t off0, uint64_t off1, int lane) {
  using V = typename ValOf<TYPE>::T;
  const uint64_t n = B.n_reads;
  const uint32_t nd = L.n_dc;
  const uint64_t stride = L.snap_stride ? L.snap_stride : L.n_ops;
  const uint64_t nops = off1 - off0;

  ReadU<DMAX> u;
  u.allmask = nd >= 32 ? 0xFFFFFFFFu : ((1u << nd) - 1u);
  const uint64_t rstride = B.per_read_clock ? n : 1, ridx = B.per_read_clock ? r : 0;
  u.spres = uniform_u32(B.read_pres[ridx]) & u.allmask;
  u.base_ignore = !B.base_ignore || B.base_ignore[r];
  u.cpres = u.base_ignore ? 0u : (uniform_u32(B.base_pres[r]) & u.allmask);
#pragma unroll
  for (int d = 0; d < DMAX; ++d) {
    u.S[d] = ((u.spres >> d) & 1u) ? uniform_u64(B.read_vc[(uint64_t)d * rstride + ridx]) : 0;
    u.C0[d] = ((u.cpres >> d) & 1u) ? uniform_u64(B.base_vc[(uint64_t)d * n + r]) : 0;
  }
  u.has_txid = B.txid && (!B.txid_valid || B.txid_valid[r]) && L.op_txid;
  u.txid = u.has_txid ? uniform_u64(B.txid[r]) : 0;

  Acc<DMAX> a;
#pragma unroll
  for (int d = 0; d < DMAX; ++d) a.mx[d] = 0;
  V v;

  const uint64_t t0 = off0 & ~(uint64_t)(OPL - 1);
  for (uint64_t g = t0 + (uint64_t)lane * OPL; g < off1; g += TILE) {
    const uint32_t meta4 = *(const uint32_t *)(L.op_meta + g);
    const u64x2 ct01 = *(const u64x2 *)(L.commit_time + g);
    const u64x2 ct23 = *(const u64x2 *)(L.commit_time + g + 2);
    uint64_t sv[OPL][DMAX];
#pragma unroll
    for (int d = 0; d < DMAX; ++d) {
      if (d < (int)nd) {
        const uint64_t *col = L.snap_vc + (uint64_t)d * stride + g;
        const u64x2 s01 = *(const u64x2 *)col;
        const u64x2 s23 = *(const u64x2 *)(col + 2);
        sv[0][d] = s01.x;
        sv[1][d] = s01.y;
        sv[2][d] = s23.x;
        sv[3][d] = s23.y;
      } else {
        sv[0][d] = sv[1][d] = sv[2][d] = sv[3][d] = 0;
      }
    }
    u32x4 sp = {u.allmask, u.allmask, u.allmask, u.allmask};
    if (L.snap_pres) sp = *(const u32x4 *)(L.snap_pres + g);
    const u64x2 p001 = *(const u64x2 *)(L.p0 + g);
    const u64x2 p023 = *(const u64x2 *)(L.p0 + g + 2);
    u64x2 p101 = {0, 0}, p123 = {0, 0};
    if (ValOf<TYPE>::NEED_P1) {
      p101 = *(const u64x2 *)(L.p1 + g);
      p123 = *(const u64x2 *)(L.p1 + g + 2);
    }
    u64x2 tx01 = {0, 0}, tx23 = {0, 0};
    if (u.has_txid) {
      tx01 = *(const u64x2 *)(L.op_txid + g);
      tx23 = *(const u64x2 *)(L.op_txid + g + 2);
    }
    const uint64_t ctv[OPL] = {ct01.x, ct01.y, ct23.x, ct23.y};
    const uint64_t p0v[OPL] = {p001.x, p001.y, p023.x, p023.y};
    const uint64_t p1v[OPL] = {p101.x, p101.y, p123.x, p123.y};
    const uint64_t txv[OPL] = {tx01.x, tx01.y, tx23.x, tx23.y};
    const uint32_t spv[OPL] = {sp.x, sp.y, sp.z, sp.w};
#pragma unroll
    for (int j = 0; j < OPL; ++j) {
      const uint64_t p = g + j;
      if (p < off0 || p >= off1) continue;
      const bool txm = u.has_txid && txv[j] == u.txid;
      if (eval_op<DMAX>(u, (uint8_t)(meta4 >> (8 * j)), ctv[j], sv[j], spv[j], txm, p, a)) v.add(p0v[j], p1v[j]);
    }
  }

  // ---- wave reduction ----
  const uint32_t count = wave_sum_u32(a.count);
  const uint32_t pres = wave_or_u32(a.pres);
  const uint32_t flags = wave_or_u32(a.flags);
  const uint64_t min_excl = wave_min_u64(a.min_excl);
  uint64_t mx[DMAX];
#pragma unroll
  for (int d = 0; d < DMAX; ++d) mx[d] = (d < (int)nd) ? wave_max_u64(a.mx[d]) : 0;

  int32_t status = (flags & FLAG_BAD) ? AM_ERR_UNEXPECTED_OPERATION : AM_OK;
  if constexpr (TYPE == AM_PN) {
    int64_t hi = v.hi;
    uint64_t lo = v.lo;
    wave_sum_i128(hi, lo);
    if (lane == 0 && status == AM_OK) {
      const int64_t b = B.base.v0 ? B.base.v0[r] : 0;
      const uint64_t s = lo + (uint64_t)b;
      hi += (b < 0 ? -1 : 0) + (s < lo ? 1 : 0);
      lo = s;
      // fits int64 iff hi is the sign extension of lo (Erlang would return a bignum)
      if (hi != ((int64_t)lo < 0 ? -1 : 0))
        status = AM_ERR_OVERFLOW;
      else
        R.value.v0[r] = (int64_t)lo;
    }
  } else if constexpr (TYPE == AM_LWW) {
    // lexicographic (has, ts, val) max across lanes
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const uint64_t wts = __shfl_xor(v.ts, o, WAVE);
      const uint64_t wval = __shfl_xor(v.val, o, WAVE);
      const bool whas = __shfl_xor((int)v.has, o, WAVE) != 0;
      const bool gt = whas && (!v.has || wts > v.ts || (wts == v.ts && wval > v.val));
      v.ts = gt ? wts : v.ts;
      v.val = gt ? wval : v.val;
      v.has = v.has || whas;
    }
    if (lane == 0 && status == AM_OK) {
      uint64_t bts = 0, bval = 0;
      uint8_t bbin = 1;  // new() = {0, <<>>}
      if (B.base.v0) {
        bts = (uint64_t)B.base.v0[r];
        bval = B.base.v1 ? B.base.v1[r] : 0;
        bbin = B.base.vflag ? B.base.vflag[r] : 0;
      }
      // erlang:max(Effect, State): the effect wins iff it sorts above the state
      const bool win = v.has && (v.ts > bts || (v.ts == bts && !bbin && v.val > bval));
      R.value.v0[r] = (int64_t)(win ? v.ts : bts);
      R.value.v1[r] = win ? v.val : bval;
      R.value.vflag[r] = win ? 0 : bbin;
    }
  }

  if (lane == 0) {
    R.status[r] = status;
    R.flags[r] = (uint8_t)(flags & 0xFFu);
    if (status == AM_OK) {
      // NewLastOp: id of the oldest excluded candidate - 1, else get_first_id/1
      const uint64_t idb = L.key_id_base ? L.key_id_base[key] : 1;
      const int64_t id_excl = L.op_id ? (int64_t)L.op_id[min_excl == NONE ? 0 : min_excl]
                                      : (int64_t)(idb + (min_excl - off0));
      const int64_t id_first = nops == 0 ? 0 : (L.op_id ? (int64_t)L.op_id[off1 - 1] : (int64_t)(idb + nops - 1));
      R.new_last_op[r] = min_excl != NONE ? id_excl - 1 : id_first;
      const bool ign = u.base_ignore && count == 0;
      const uint32_t opres = ign ? 0u : (pres | u.cpres);
      R.last_ct_ignore[r] = ign ? 1 : 0;
      R.last_ct_pres[r] = opres;
#pragma unroll
      for (int d = 0; d < DMAX; ++d) {
        if (d < (int)nd) {
          const uint64_t m = mx[d] > u.C0[d] ? mx[d] : u.C0[d];
          R.last_ct[(uint64_t)d * n + r] = ((opres >> d) & 1u) ? m : 0;
        }
      }
      R.is_new_ss[r] = count > 0;
      R.count[r] = count;
    }
  }
}

// TYPE_HINT != 0: every read of the batch has that type; 0: per-read switch.
template <int DMAX, int TYPE_HINT>
__global__ void __launch_bounds__(BLOCK) k_materialize_scalar(am_op_log L, am_read_batch B, am_read_result R) {
  const int lane = threadIdx.x & (WAVE - 1);
  const uint32_t wave_in_block = uniform_u32(threadIdx.x >> 6);
  const uint64_t n = B.n_reads;
  const uint64_t waves_total = (uint64_t)gridDim.x * WPB;

  for (uint64_t r = (uint64_t)blockIdx.x * WPB + wave_in_block; r < n; r += waves_total) {
    const uint64_t key = uniform_u64(B.key[r]);
    const uint32_t type = TYPE_HINT ? (uint32_t)TYPE_HINT : uniform_u32(B.type[r]);
    if (key >= L.n_keys) {
      if (lane == 0) R.status[r] = AM_ERR_INVALID;
      continue;
    }
    const uint64_t off0 = uniform_u64(L.key_off[key]);
    const uint64_t off1 = uniform_u64(L.key_off[key + 1]);
    const uint32_t ktype = uniform_u32(L.key_type[key]);
    const uint32_t kflags = L.key_flags ? uniform_u32(L.key_flags[key]) : 0u;
    const uint32_t rtype = TYPE_HINT ? uniform_u32(B.type[r]) : type;
    if (off1 > off0 && (ktype != rtype || (kflags & AM_KEY_MIXED_TYPES))) {
      if (lane == 0) R.status[r] = AM_ERR_CORRUPTED_OPS_CACHE;  // erlang:error(corrupted_ops_cache)
      continue;
    }
    if (TYPE_HINT && rtype != (uint32_t)TYPE_HINT) {
      if (lane == 0) R.status[r] = AM_ERR_INVALID;
      continue;
    }
    if constexpr (TYPE_HINT == AM_PN) {
      read_scalar<DMAX, AM_PN>(L, B, R, r, key, off0, off1, lane);
    } else if constexpr (TYPE_HINT == AM_LWW) {
      read_scalar<DMAX, AM_LWW>(L, B, R, r, key, off0, off1, lane);
    } else {
      switch (type) {
        case AM_PN: read_scalar<DMAX, AM_PN>(L, B, R, r, key, off0, off1, lane); break;
        case AM_LWW: read_scalar<DMAX, AM_LWW>(L, B, R, r, key, off0, off1, lane); break;
        default:
          if (lane == 0) R.status[r] = AM_ERR_UNSUPPORTED;
      }
    }
  }
}

template <int HINT>
int launch_hint(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R) {
  uint64_t blocks = (B->n_reads + WPB - 1) / WPB;
  const uint64_t cap = (uint64_t)ctx->n_cu * 32;
  if (blocks > cap) blocks = cap;
  if (blocks == 0) return AM_OK;
  dim3 grid((unsigned)blocks), block(BLOCK);
  const uint32_t nd = L->n_dc;
#define AM_LAUNCH(D)                                                                                 \
  hipLaunchKernelGGL((k_materialize_scalar<D, HINT>), grid, block, 0, ctx->stream, *L, *B, *R); \
  break;
  switch (nd <= 1 ? 1 : nd <= 2 ? 2 : nd <= 3 ? 3 : nd <= 4 ? 4 : nd <= 8 ? 8 : nd <= 16 ? 16 : 32) {
    case 1: AM_LAUNCH(1)
    case 2: AM_LAUNCH(2)
    case 3: AM_LAUNCH(3)
    case 4: AM_LAUNCH(4)
    case 8: AM_LAUNCH(8)
    case 16: AM_LAUNCH(16)
    default: AM_LAUNCH(32)
  }
#undef AM_LAUNCH
  AM_HIP(hipGetLastError());
  return AM_OK;
}

}  // namespace

// The one-read-per-wave kernel (PN, LWW): kept for A/B comparisons (AM_KERNEL=scalar).
int am_launch_scalar(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R) {
  switch (B->type_hint) {
    case AM_PN: return launch_hint<AM_PN>(ctx, L, B, R);
    case AM_LWW: return launch_hint<AM_LWW>(ctx, L, B, R);
    case 0: return launch_hint<0>(ctx, L, B, R);
    default:
      am_set_error("the scalar kernel handles PN and LWW only");
      return AM_ERR_UNSUPPORTED;
  }
}
