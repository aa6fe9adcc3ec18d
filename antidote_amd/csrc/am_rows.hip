// am_rows.hip -- materialize/4 for SHORT op logs: one 16-lane DPP row per read.
//
// A riak_core partition's keys are mostly short-lived or cold: the mixed (C4, 16 ops
// per key) and Zipf (C5, 95% of keys with <= 48 ops) workloads are dominated by reads
// whose whole log is a few cache lines.  Giving such a read a wavefront (k_stream) or a
// workgroup (k_sets) leaves most lanes idle and pays a full wave/block reduction per
// read.  Here each wavefront takes a batch of 64 consecutive reads and splits into four
// 16-lane rows; row q owns reads 16q .. 16q+15 of the batch and walks them one after
// another, 16 ops per step (one op per lane, a contiguous 128-byte segment per column
// per row).  Per-read results come from DPP row butterflies (4 steps, no readlane), and
// read 16q+s's results are parked in lane 16q+s -- so, as in k_stream, the batch's
// results leave with one coalesced store per output column.
//
// Types:
//   PN counter / LWW register  commutative reductions in registers (am_wave.h)
//   bounded counter            n_dc <= 16: every included amount goes into the row's LDS
//                              slot array with one 64-bit LDS atomic (exact: a row read has
//                              <= 127 entries, each below 2^56 -- a larger amount defers the
//                              read to the workgroup tier), then lane s writes slots s,
//                              s+16, ... with the base added in 128 bits; n_dc > 16: the
//                              (slot, amount) pairs go to an LDS list that each lane scans
//                              for its slots
// (short add-wins-set / MV-register reads have their own row kernel, am_group.hip).
// A read longer than the short limit, or whose entries do not fit the row's LDS list, is
// handed to the workgroup tier (k_stream for PN/LWW skips it on its own; the bounded
// counter gets it through a hand-off list).
#include "am_block.h"

using namespace amk;

namespace {

constexpr int BLOCK = 256;
constexpr int WPB = BLOCK / WAVE;
constexpr int G = 16;
constexpr uint32_t RK = 64;  // bounded counter: (slot, amount) entries per row

template <int DMAX>
struct RowSmem {
  static constexpr bool SLOTS = DMAX <= 16;                            // slot-array mode
  static constexpr uint32_t NS = SLOTS ? DMAX * DMAX + DMAX : 1;      // P then D slots
  static constexpr uint32_t NL = SLOTS ? 1 : RK;                      // list mode entries
  uint64_t acc[NS];        // slot sums (slot-array mode)
  uint32_t pres[(NS + 31) / 32];
  uint64_t ka[NL];         // amount (list mode)
  int32_t kp[NL];          // slot (list mode)
  uint32_t ctr[4];         // [0] entries [2] overflow of a slot sum [3] list overflow / big amount
};

template <int TYPE>
struct RowVal {  // per-lane value accumulator of the scalar types (unused for the others)
  using T = PnVal;
};
template <>
struct RowVal<AM_LWW> {
  using T = LwwVal;
};

template <int DMAX>
struct ROut {  // per-lane buffered outputs of read (batch base + lane)
  int32_t status;
  uint32_t flags, pres, count, ign, newss, vflag, store;
  int64_t nlo;
  uint64_t ct[DMAX];
  uint64_t v0, v1;
};

// (at D = 16 the compiler takes ~350 VGPRs, one wave per SIMD; asked for two it fits 224
// without spilling, but C5's bounded-counter rows then ran 2.1x slower: DESIGN.md 8)

template <int DMAX, int TYPE, bool GENERAL, bool PACKED>
__global__ void __launch_bounds__(BLOCK) k_rows(am_op_log L, am_read_batch B, am_read_result R, am_sel S,
                                                am_rows_cfg C) {
  constexpr bool BC = TYPE == AM_BCOUNTER;
  constexpr bool LDS = BC;
  using V = typename RowVal<TYPE>::T;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  using RS = RowSmem<DMAX>;
  RS *rs = LDS ? ((RS *)smem_raw) + (threadIdx.x / G) : nullptr;

  const uint32_t lane = threadIdx.x & (WAVE - 1);
  const uint32_t row = lane / G, sl = lane % G;
  const uint64_t n = B.n_reads;
  const uint32_t sel0 = S.idx ? uniform_u32(S.range[0]) : 0u;
  const uint64_t nsel = S.idx ? (uint64_t)(uniform_u32(S.range[1]) - sel0) : n;
  const uint32_t *sbase = S.idx ? S.idx + sel0 : nullptr;
  const uint32_t nd = L.n_dc;
  const uint32_t np = nd * nd, nslot = np + nd;
  const uint64_t stride = L.snap_stride ? L.snap_stride : L.n_ops;
  const uint64_t W = (uint64_t)gridDim.x * WPB;
  const uint64_t gw = (uint64_t)blockIdx.x * WPB + uniform_u32(threadIdx.x >> 6);
  const uint64_t n_batches = (nsel + WAVE - 1) / WAVE;
  const uint32_t allmask = nd >= 32 ? 0xFFFFFFFFu : ((1u << nd) - 1u);

  // batch-uniform read clock (per-read clocks are loaded per read below)
  ReadU<DMAX> u;
  u.allmask = allmask;
  u.base_ignore = true, u.has_txid = false, u.txid = 0, u.cpres = 0;
#pragma unroll
  for (int d = 0; d < DMAX; ++d) u.C0[d] = 0;
  if (!GENERAL || !B.per_read_clock) {
    u.spres = uniform_u32(B.read_pres[0]) & allmask;
#pragma unroll
    for (int d = 0; d < DMAX; ++d)
      u.S[d] = (d < (int)nd && ((u.spres >> d) & 1u)) ? uniform_u64(B.read_vc[d]) : 0;
  }

  for (uint64_t bid = gw; bid < n_batches; bid += W) {
    // ---- batch metadata: lane i <-> read rb + i ----
    const uint64_t rb = bid * WAVE;
    const uint32_t nb = (uint32_t)(nsel - rb < (uint64_t)WAVE ? nsel - rb : (uint64_t)WAVE);
    const uint64_t bmask = C.mask ? uniform_u64(C.mask[bid]) : ~0ull;  // k_stream's hand-off
    if (!bmask) continue;
    uint64_t key = 0, off0 = 0, off1 = 0, r = 0, tb = 0;  // tb: the key's packed time base
    int32_t st = AM_OK;
    if (lane < nb && ((bmask >> lane) & 1u)) {
      r = sbase ? (uint64_t)sbase[rb + lane] : rb + lane;
      key = B.key[r];
      const uint32_t rtype = B.type[r];
      if (key >= L.n_keys) {
        st = AM_ERR_INVALID;
      } else {
        off0 = L.key_off[key];
        off1 = am_kend(L, key);
        if (PACKED) tb = L.key_tbase[key];  // with the batch's metadata, not per read start
        const uint32_t ktype = L.key_type[key];
        const uint32_t kfl = L.key_flags ? (uint32_t)L.key_flags[key] : 0u;
        if (off1 > off0 && (ktype != rtype || (kfl & AM_KEY_MIXED_TYPES)))
          st = AM_ERR_CORRUPTED_OPS_CACHE;  // erlang:error(corrupted_ops_cache)
        else if (rtype != (uint32_t)TYPE)
          st = AM_ERR_INVALID;
      }
      if (st != AM_OK) off1 = off0;
    }
    const uint64_t len = off1 - off0;
    const bool mine = lane < nb && ((bmask >> lane) & 1u) && len <= C.short_max;  // error reads have len 0
    // bounded counter: long reads go to the workgroup tier through the hand-off list
    if (C.list) {
      const bool hand = lane < nb && !mine;
      const uint64_t hm = __ballot(hand);
      if (hm) {
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(C.count, (uint32_t)__popcll(hm));
        base = uniform_u32(base);
        if (hand) C.list[base + __popcll(hm & ((1ull << lane) - 1))] = (uint32_t)r;
      }
    }

    // ---- per-lane buffered result, initialised to materialize/4 of an empty log ----
    ROut<DMAX> o;
    o.status = st, o.store = mine ? 1u : 0u;
    o.flags = 0, o.pres = 0, o.count = 0, o.ign = 1, o.newss = 0, o.nlo = 0;
#pragma unroll
    for (int d = 0; d < DMAX; ++d) o.ct[d] = 0;
    o.v0 = 0, o.v1 = 0, o.vflag = TYPE == AM_LWW ? 1 : 0;
    if (GENERAL && mine) {
      if (B.base_ignore && !B.base_ignore[r]) {
        o.ign = 0;
        o.pres = B.base_pres[r] & allmask;
#pragma unroll
        for (int d = 0; d < DMAX; ++d)
          if (d < (int)nd && ((o.pres >> d) & 1u)) o.ct[d] = B.base_vc[(uint64_t)d * n + r];
      }
      if ((TYPE == AM_PN || TYPE == AM_LWW) && B.base.v0) {
        o.v0 = (uint64_t)B.base.v0[r];
        if (TYPE == AM_LWW) {
          o.v1 = B.base.v1 ? B.base.v1[r] : 0;
          o.vflag = B.base.vflag ? B.base.vflag[r] : 0;
        }
      }
    }
    // An empty log still returns the base value: bcounters copy the base slots
    // (materialize/4 on [] applies no effect).  Done by the row below as a read with zero
    // ops, so the value paths stay in one place.
    const bool work = mine && st == AM_OK && (len > 0 || LDS);
    const uint64_t wmask = __ballot(work);
    if (wmask) {
      uint32_t rowbits = (uint32_t)((wmask >> (row * G)) & 0xFFFFu);
      uint32_t s = rowbits ? (uint32_t)__builtin_ctz(rowbits) : 16u;
      // current read of the row (row-uniform values)
      uint64_t o0 = 0, o1 = 0, rj = 0, keyj = 0, t = 0;
      Acc<DMAX> a;
      AccP<DMAX> ap;
      PkRead<DMAX> pk;
      V v;
      a.reset();
      ap.reset();
      v.reset();
      // (re)start the row's current read; uniform call (the shuffles need every lane),
      // takes effect in rows with upd set; rows with s == 16 are idle
      auto begin = [&](bool upd) {
        const uint32_t j = row * G + (s < 16 ? s : 0);
        const uint64_t n0 = shfl_u64(off0, j), n1 = shfl_u64(off1, j), nr = shfl_u64(r, j), nk = shfl_u64(key, j);
        const uint64_t ntb = PACKED ? shfl_u64(tb, j) : 0;
        if (!upd) return;
        o0 = n0, o1 = n1, rj = nr, keyj = nk;
        t = 0;
        if (s >= 16) return;
        if (GENERAL) {
          if (B.per_read_clock) {
            u.spres = B.read_pres[rj] & allmask;
#pragma unroll
            for (int d = 0; d < DMAX; ++d)
              u.S[d] = (d < (int)nd && ((u.spres >> d) & 1u)) ? B.read_vc[(uint64_t)d * n + rj] : 0;
          }
          u.base_ignore = !B.base_ignore || B.base_ignore[rj];
          u.cpres = u.base_ignore ? 0u : (B.base_pres[rj] & allmask);
#pragma unroll
          for (int d = 0; d < DMAX; ++d)
            u.C0[d] = (d < (int)nd && ((u.cpres >> d) & 1u)) ? B.base_vc[(uint64_t)d * n + rj] : 0;
          u.has_txid = B.txid && (!B.txid_valid || B.txid_valid[rj]) && L.op_txid;
          u.txid = u.has_txid ? B.txid[rj] : 0;
        }
        if (PACKED) pk_setup(u, nd, ntb, pk);
        if (LDS) {
          if (sl == 0) rs->ctr[0] = 0, rs->ctr[1] = 0, rs->ctr[2] = 0, rs->ctr[3] = 0;
          if (RS::SLOTS) {
            for (uint32_t i = sl; i < nslot; i += G) rs->acc[i] = 0;
            for (uint32_t i = sl; i < (nslot + 31) / 32; i += G) rs->pres[i] = 0;
          }
          wave_sync();
        }
      };
      begin(true);
      // one op's streamed columns, loaded one step ahead of their use
      struct ROp {
        uint64_t w;         // full: commit_time
        uint32_t meta, sp;  // op_meta (full view, bounded counter); snapshot presence
        uint32_t x[DMAX];   // packed: X[d] - key_tbase
        uint64_t sv[DMAX];  // full: snapshot entries
        uint64_t tx, p0, p1;
      };
      auto load_op = [&](ROp &q, uint64_t p, bool valid) {
        if (!valid) return;
        if (PACKED) {
#pragma unroll
          for (int d = 0; d < DMAX; ++d) q.x[d] = d < (int)nd ? L.pk_vc[(uint64_t)d * stride + p] : 0u;
          if (BC) q.meta = L.op_meta[p];
        } else {
          q.meta = L.op_meta[p];
          q.w = L.commit_time[p];
#pragma unroll
          for (int d = 0; d < DMAX; ++d) q.sv[d] = d < (int)nd ? L.snap_vc[(uint64_t)d * stride + p] : 0;
        }
        q.sp = (GENERAL && L.snap_pres) ? L.snap_pres[p] : allmask;
        q.tx = (GENERAL && u.has_txid) ? L.op_txid[p] : 0;
        q.p0 = L.p0[p];
        if (TYPE != AM_PN) q.p1 = L.p1[p];
      };
      ROp cur, nxt;
      load_op(cur, o0 + sl, s < 16 && o0 + sl < o1);
      while (__ballot(s < 16)) {
        const bool act = s < 16;
        const uint64_t p = o0 + t + sl;
        const bool fin_next = act && o0 + t + G >= o1;
        {  // prefetch the next step: this read at t + G, or the row's next read
          const uint32_t rest = act ? (rowbits & ~(1u << s)) : 0u;
          const uint32_t s2 = rest ? (uint32_t)__builtin_ctz(rest) : 16u;
          const uint32_t j2 = row * G + (s2 < 16 ? s2 : 0);
          const uint64_t n0 = shfl_u64(off0, j2), n1 = shfl_u64(off1, j2);
          if (fin_next) load_op(nxt, n0 + sl, s2 < 16 && n0 + sl < n1);
          else load_op(nxt, p + G, act && p + G < o1);
        }
        if (act && p < o1) {
          // ---- one op: is_op_in_snapshot/7 + the type's effect ----
          uint32_t meta = PACKED && !BC ? 0u : cur.meta;
          const bool txm = GENERAL && u.has_txid && cur.tx == u.txid;
          bool in;
          if (PACKED && cur.x[0] != AM_PK_ESC) {
            in = pk_eval<DMAX, GENERAL>(pk, u, cur.x, txm, p, ap);
          } else {
            uint64_t ct, sv[DMAX];
            if (PACKED) {  // rare: the op does not fit the packed view
              esc_load<DMAX>(L, nd, stride, p, sv, ct, meta);
            } else {
              ct = cur.w;
#pragma unroll
              for (int d = 0; d < DMAX; ++d) sv[d] = cur.sv[d];
            }
            in = eval_op<DMAX, GENERAL>(u, meta, ct, sv, cur.sp, txm, p, a);
          }
          if (in && !(LDS && (meta & AM_META_BAD))) {
            if constexpr (TYPE == AM_PN || TYPE == AM_LWW) {
              v.add(cur.p0, TYPE == AM_LWW ? cur.p1 : 0);
            } else if constexpr (BC) {
              const uint32_t kind = AM_META_KIND(meta);
              const uint32_t from = (uint32_t)(cur.p1 & 0xFF), to = (uint32_t)((cur.p1 >> 8) & 0xFF);
              if (kind <= AM_BC_TRANSFER && from < nd && to < nd) {
                const uint32_t slot =
                    kind == AM_BC_DECREMENT ? np + from : from * nd + (kind == AM_BC_INCREMENT ? from : to);
                if (RS::SLOTS) {
                  const int64_t x = (int64_t)cur.p0;
                  if (x >= (1ll << 56) || x < -(1ll << 56)) {
                    rs->ctr[3] = 1;  // exactness of the 64-bit sums not guaranteed: defer
                  } else {
                    atomicAdd((unsigned long long *)&rs->acc[slot], (unsigned long long)cur.p0);
                    atomicOr(&rs->pres[slot >> 5], 1u << (slot & 31));
                  }
                } else {
                  const uint32_t e = atomicAdd(&rs->ctr[0], 1u);
                  if (e < RK) rs->ka[e] = cur.p0, rs->kp[e] = (int32_t)slot;
                  else rs->ctr[3] = 1;
                }
              } else {
                a.flags |= FLAG_BAD;
              }
            }
          }
        }
        t += G;
        const bool fin = act && o0 + t >= o1;
        if (__ballot(fin)) {
          // ---- row reductions (full EXEC), then rows that finished a read emit it ----
          if (PACKED) {  // rows still inside a read keep their partials until they finish
            Acc<DMAX> af = a;
            pk_fold(ap, pk.K, u.allmask, af);
            if (fin) a = af, ap.reset();
          }
          const uint32_t count = row_sum_u32(a.count);
          const uint32_t flags = row_or_u32(a.flags);
          const uint32_t pres = row_or_u32(a.pres);
          const uint64_t min_excl = row_min_u64(a.min_excl);
          uint64_t mx[DMAX];
#pragma unroll
          for (int d = 0; d < DMAX; ++d) mx[d] = d < (int)nd ? row_max_u64(a.mx[d]) : 0;
          V vr = v;  // rows still inside a read keep their per-lane partials
          if constexpr (TYPE == AM_PN) row_sum_i128(vr.hi, vr.lo);
          if constexpr (TYPE == AM_LWW) row_max_lww(vr);
          wave_sync();
          if (fin) {
            const uint32_t j = row * G + s;
            int32_t status = (flags & FLAG_BAD) ? AM_ERR_UNEXPECTED_OPERATION : AM_OK;
            bool defer = false;
            uint64_t v0 = 0, v1 = 0;
            uint32_t vflag = 0;
            if constexpr (TYPE == AM_PN) {
              int64_t hi = vr.hi;
              uint64_t lo = vr.lo;
              const int64_t b = (GENERAL && B.base.v0) ? B.base.v0[rj] : 0;
              add128(hi, lo, b < 0 ? -1 : 0, (uint64_t)b);
              if (status == AM_OK && hi != ((int64_t)lo < 0 ? -1 : 0)) status = AM_ERR_OVERFLOW;
              v0 = lo;
            } else if constexpr (TYPE == AM_LWW) {
              uint64_t bts = 0, bval = 0;
              uint32_t bbin = 1;  // new() = {0, <<>>}
              if (GENERAL && B.base.v0) {
                bts = (uint64_t)B.base.v0[rj];
                bval = B.base.v1 ? B.base.v1[rj] : 0;
                bbin = B.base.vflag ? B.base.vflag[rj] : 0;
              }
              const bool win = vr.has && (vr.ts > bts || (vr.ts == bts && !bbin && vr.val > bval));
              v0 = win ? vr.ts : bts;
              v1 = win ? vr.val : bval;
              vflag = win ? 0 : bbin;
            } else if constexpr (BC) {
              if (status == AM_OK && rs->ctr[3]) defer = true;
              if (RS::SLOTS && status == AM_OK && !defer) {
                // |row sum| < 127 * 2^56 < 2^63: exact in int64; the base is added in 128 bits
                auto total = [&](uint32_t i, int64_t &hi, uint64_t &lo, uint32_t &pr) {
                  uint32_t bp = 0;
                  const int64_t bv = GENERAL ? bc_base(B, rj, np, nd, i, bp) : 0;
                  const int64_t x = (int64_t)rs->acc[i];
                  hi = bv < 0 ? -1 : 0, lo = (uint64_t)bv;
                  add128(hi, lo, x < 0 ? -1 : 0, (uint64_t)x);
                  pr = bp | ((rs->pres[i >> 5] >> (i & 31)) & 1u);
                };
                uint32_t ovf = 0;
                if (GENERAL && B.base.set_off)
                  for (uint32_t i = sl; i < nslot; i += G) {
                    int64_t hi;
                    uint64_t lo;
                    uint32_t pr;
                    total(i, hi, lo, pr);
                    ovf |= hi != ((int64_t)lo < 0 ? -1 : 0) ? 1u : 0u;
                  }
                if (row_or_u32(ovf)) {
                  status = AM_ERR_OVERFLOW;
                } else {  // the present slots as (slot, value) pairs: the P / D orddicts' entries
                  // (a slot's place = the present slots below it, popcounts of the row's bitmap)
                  if (GENERAL && B.base.set_off) {
                    for (uint32_t i = sl; i < nslot; i += G) {
                      uint32_t bp = 0;
                      (void)bc_base(B, rj, np, nd, i, bp);
                      if (bp) atomicOr(&rs->pres[i >> 5], 1u << (i & 31));
                    }
                    wave_sync();
                  }
                  // chunk c = slots [16c, 16c + 16), lane sl slot 16c + sl: the chunk's 16 bits
                  // are one half of a bitmap word (the same word for the whole row)
                  const uint64_t so = R.value.set_off[rj], cap = R.value.set_off[rj + 1] - so;
                  uint32_t ne = 0;
                  if constexpr (!GENERAL) {
                    // every LDS read of the emit issued up front (one exposed latency at one
                    // wave per SIMD, not one per chunk); no base: a slot's value is its sum
                    constexpr uint32_t NC = (RS::NS + G - 1) / G, NWD = (RS::NS + 31) / 32;
                    uint32_t pw[NWD];
                    uint64_t av[NC];
#pragma unroll
                    for (uint32_t w = 0; w < NWD; ++w) pw[w] = w < (nslot + 31) / 32 ? rs->pres[w] : 0u;
#pragma unroll
                    for (uint32_t c = 0; c < NC; ++c) av[c] = c * G + sl < nslot ? rs->acc[c * G + sl] : 0ull;
#pragma unroll
                    for (uint32_t c = 0; c < NC; ++c) {
                      const uint32_t bits = (pw[c >> 1] >> ((c & 1u) * 16u)) & 0xFFFFu;
                      const uint32_t i = c * G + sl;
                      const uint32_t rank = ne + (uint32_t)__popc(bits & ((1u << sl) - 1u));
                      if (i < nslot && ((bits >> sl) & 1u) && rank < cap) {
                        R.value.set_a[so + rank] = i;
                        R.value.set_b[so + rank] = av[c];
                      }
                      ne += (uint32_t)__popc(bits);
                    }
                  }
                  for (uint32_t c = 0; GENERAL && c * G < nslot; ++c) {
                    const uint32_t bits = (rs->pres[c >> 1] >> ((c & 1u) * 16u)) & 0xFFFFu;
                    const uint32_t i = c * G + sl;
                    const uint32_t rank = ne + (uint32_t)__popc(bits & ((1u << sl) - 1u));
                    if (i < nslot && ((bits >> sl) & 1u) && rank < cap) {
                      int64_t hi;
                      uint64_t lo;
                      uint32_t pr;
                      total(i, hi, lo, pr);
                      R.value.set_a[so + rank] = i;
                      R.value.set_b[so + rank] = lo;
                    }
                    ne += (uint32_t)__popc(bits);
                  }
                  if (ne > cap) status = AM_ERR_CAPACITY;
                  v0 = ne;
                }
              } else if (status == AM_OK && !defer) {
                const uint32_t ne = rs->ctr[0];
                const uint32_t ne4 = (ne + 3) & ~3u;
                if (sl < ne4 - ne) rs->kp[ne + sl] = -1;  // pad the slot list to whole int4 loads
                // With every |amount| < 2^56 (and no base values) the <= 64 entries of a
                // slot cannot leave int64: the exact overflow pass is skipped.
                uint32_t big = (GENERAL && B.base.set_off) ? 1u : 0u;
                for (uint32_t e = sl; e < ne; e += G) {
                  const int64_t x = (int64_t)rs->ka[e];
                  big |= (x >= (1ll << 56) || x < -(1ll << 56)) ? 1u : 0u;
                }
                big = row_or_u32(big);
                wave_sync();
                // sum of the row's entries with slot i (int4 loads of the slot list)
                auto slot_sum = [&](uint32_t i, int64_t &hi, uint64_t &lo) -> uint32_t {
                  uint32_t hit = 0;
                  const int4 *kp4 = reinterpret_cast<const int4 *>(rs->kp);
#pragma unroll 4
                  for (uint32_t e = 0; e < ne4; e += 4) {
                    const int4 k = kp4[e >> 2];
                    const int32_t ks[4] = {k.x, k.y, k.z, k.w};
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                      if (ks[q] == (int32_t)i) {
                        const int64_t x = (int64_t)rs->ka[e + q];
                        add128(hi, lo, x < 0 ? -1 : 0, (uint64_t)x);
                        hit = 1;
                      }
                  }
                  return hit;
                };
                auto base_of = [&](uint32_t i, uint32_t &bpres) -> int64_t {
                  bpres = 0;
                  if (!GENERAL) return 0;
                  return bc_base(B, rj, np, nd, i, bpres);
                };
                if (big) {  // pass 1: exact 128-bit sums of the lane's slots, overflow check
                  uint32_t ovf = 0;
                  for (uint32_t i = sl; i < nslot; i += G) {
                    uint32_t bp;
                    const int64_t bv = base_of(i, bp);
                    int64_t hi = bv < 0 ? -1 : 0;
                    uint64_t lo = (uint64_t)bv;
                    slot_sum(i, hi, lo);
                    if (hi != ((int64_t)lo < 0 ? -1 : 0)) ovf = 1;
                  }
                  if (ovf) atomicOr(&rs->ctr[2], 1u);
                  wave_sync();
                }
                if (big && rs->ctr[2]) {
                  status = AM_ERR_OVERFLOW;
                } else {  // the present slots as (slot, value) pairs
                  const uint32_t ne = bc_emit<G>(R, rj, nslot, sl, row * G, [&](uint32_t i, int64_t &x) {
                    uint32_t bpres;
                    const int64_t bv = base_of(i, bpres);
                    int64_t hi = bv < 0 ? -1 : 0;
                    uint64_t lo = (uint64_t)bv;
                    bpres |= slot_sum(i, hi, lo);
                    x = (int64_t)lo;
                    return bpres != 0;
                  });
                  if (ne > R.value.set_off[rj + 1] - R.value.set_off[rj]) status = AM_ERR_CAPACITY;
                  v0 = ne;
                }
              }
            }
            // NewLastOp: id of the oldest excluded candidate - 1, else get_first_id/1
            const uint64_t nops = o1 - o0;
            const uint64_t idb = L.key_id_base ? L.key_id_base[keyj] : 1;
            int64_t nlo;
            if (min_excl != NONE)
              nlo = ((GENERAL && L.op_id) ? (int64_t)L.op_id[min_excl] : (int64_t)(idb + (min_excl - o0))) - 1;
            else if (nops == 0)
              nlo = 0;
            else
              nlo = (GENERAL && L.op_id) ? (int64_t)L.op_id[o1 - 1] : (int64_t)(idb + nops - 1);
            const bool ign = u.base_ignore && count == 0;
            const uint32_t opres = ign ? 0u : (pres | u.cpres);
            if (defer && sl == 0) C.list[atomicAdd(C.count, 1u)] = (uint32_t)rj;
            if (lane == j) {
              o.store = defer ? 0u : 1u;
              o.status = status;
              o.flags = flags & 0xFFu;
              o.count = count;
              o.pres = opres;
              o.ign = ign ? 1 : 0;
              o.newss = count > 0;
              o.nlo = nlo;
#pragma unroll
              for (int d = 0; d < DMAX; ++d) {
                const uint64_t m = mx[d] > u.C0[d] ? mx[d] : u.C0[d];
                o.ct[d] = ((opres >> d) & 1u) ? m : 0;
              }
              o.v0 = v0, o.v1 = v1, o.vflag = vflag;
            }
            a.reset();
            v.reset();
            rowbits &= ~(1u << s);
            s = rowbits ? (uint32_t)__builtin_ctz(rowbits) : 16u;
          }
          wave_sync();
          begin(fin);
        }
        cur = nxt;
      }
    }
    // ---- the batch's results: one coalesced store per column ----
    if (lane < nb && o.store) {
      R.status[r] = o.status;
      if (o.status == AM_OK) {
        R.flags[r] = (uint8_t)o.flags;
        R.new_last_op[r] = o.nlo;
        R.last_ct_ignore[r] = (uint8_t)o.ign;
        R.last_ct_pres[r] = o.pres;
#pragma unroll
        for (int d = 0; d < DMAX; ++d)
          if (d < (int)nd) R.last_ct[(uint64_t)d * n + r] = o.ct[d];
        R.is_new_ss[r] = (uint8_t)o.newss;
        R.count[r] = o.count;
        if (TYPE == AM_PN || TYPE == AM_LWW) R.value.v0[r] = (int64_t)o.v0;
        if (TYPE == AM_BCOUNTER) R.value.set_len[r] = (uint32_t)o.v0;  // the entry count
        if (TYPE == AM_LWW) {
          R.value.v1[r] = o.v1;
          R.value.vflag[r] = (uint8_t)o.vflag;
        }
      }
    }
  }
}

template <int D, int TYPE, bool GENERAL, bool PACKED>
int launch_d(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S,
             const am_rows_cfg &C) {
  constexpr bool LDS = TYPE == AM_BCOUNTER;
  const size_t smem = LDS ? sizeof(RowSmem<D>) * (BLOCK / G) : 0;
  static int occ = 0;
  if (occ == 0) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_rows<D, TYPE, GENERAL, PACKED>, BLOCK, smem) != hipSuccess ||
        nb <= 0)
      nb = 2;
    occ = nb;
  }
  const uint64_t batches = (B->n_reads + WAVE - 1) / WAVE;
  uint64_t blocks = (batches + WPB - 1) / WPB;
  const uint64_t cap = (uint64_t)ctx->n_cu * (uint64_t)occ;
  if (blocks > cap) blocks = cap;
  if (blocks == 0) return AM_OK;
  hipLaunchKernelGGL((k_rows<D, TYPE, GENERAL, PACKED>), dim3((unsigned)blocks), dim3(BLOCK), smem, ctx->stream, *L, *B,
                     *R, S, C);
  AM_HIP(hipGetLastError());
  return AM_OK;
}

template <int TYPE, bool GENERAL, bool PACKED>
int launch(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S,
           const am_rows_cfg &C) {
  const uint32_t nd = L->n_dc;
  if (nd <= 1) return launch_d<1, TYPE, GENERAL, PACKED>(ctx, L, B, R, S, C);
  if (nd <= 2) return launch_d<2, TYPE, GENERAL, PACKED>(ctx, L, B, R, S, C);
  if (nd <= 3) return launch_d<3, TYPE, GENERAL, PACKED>(ctx, L, B, R, S, C);
  if (nd <= 4) return launch_d<4, TYPE, GENERAL, PACKED>(ctx, L, B, R, S, C);
  if (nd <= 8) return launch_d<8, TYPE, GENERAL, PACKED>(ctx, L, B, R, S, C);
  if (nd <= 16) return launch_d<16, TYPE, GENERAL, PACKED>(ctx, L, B, R, S, C);
  return launch_d<32, TYPE, GENERAL, PACKED>(ctx, L, B, R, S, C);
}

template <int TYPE>
int launch_t(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S,
             const am_rows_cfg &C) {
  const bool general = am_batch_general(L, B);
  const bool packed = am_log_packed(L);
  if (general) return packed ? launch<TYPE, true, true>(ctx, L, B, R, S, C) : launch<TYPE, true, false>(ctx, L, B, R, S, C);
  return packed ? launch<TYPE, false, true>(ctx, L, B, R, S, C) : launch<TYPE, false, false>(ctx, L, B, R, S, C);
}

}  // namespace

int am_launch_rows(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S, uint32_t type,
                   const am_rows_cfg &C) {
  switch (type) {
    case AM_PN: return launch_t<AM_PN>(ctx, L, B, R, S, C);
    case AM_LWW: return launch_t<AM_LWW>(ctx, L, B, R, S, C);
    case AM_BCOUNTER: return launch_t<AM_BCOUNTER>(ctx, L, B, R, S, C);
    default: return AM_ERR_UNSUPPORTED;
  }
}
