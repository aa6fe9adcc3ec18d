// am_big.hip -- materialize/4 for add-wins-set / MV-register reads beyond the LDS
// tier: Zipf-hot keys with up to 2^20+ ops, whose births/kills cannot be held by one
// workgroup (am_sets.hip hands them over through its retry list).
//
// The closed form of am_sets.hip still holds -- a birth (a, b) at position p survives
// iff no kill with the same kill key (AW: (tok, elem); MV: tok) sits at q > p -- but it
// is evaluated across many workgroups:
//   k_big_prep      one thread per big read: its op range, record capacity, chunk count
//   k_big_offsets   one workgroup: exclusive scans -> chunk / record / hash offsets
//   k_big_chunk     one workgroup per 1024-op chunk of any big read (flattened, so a hot
//                   key spreads over the whole GPU): inclusion test + scalar partials
//                   (global atomics), births/kills in LDS, LOCAL resolution (a birth
//                   killed later in the same chunk is dead for good), then exports the
//                   chunk's surviving births and its kills (one per kill key: the
//                   latest) to global records.  A kill only matters for births at
//                   earlier positions, so nothing else crosses chunks.
//   k_big_hash      exported births -> per-read open-addressing hash on the kill key
//   k_big_kill      each exported kill probes the hash: same key, earlier birth -> dead
//   k_big_finish    one workgroup per big read: survivors sorted into the reference's
//                   order (LDS, or global scratch when they do not fit) -- AW: elem, newest
//                   birth first, the effect's token order, base tokens last; MV: (value,
//                   token), de-duplicated -- CSR + scalar outputs
// Chunk-local resolution makes the global traffic proportional to what escapes a chunk:
// for the MV register's override chain that is about one birth per chunk.
// Bounded counters (keyed sums) use the same chunking: per-chunk LDS slot sums, flushed
// into per-read global 128-bit slots (64-bit atomics + carry), checked and written by
// k_big_finish -- a hot key no longer serializes on one workgroup.
#include "am_block.h"

using namespace amk;

namespace {

constexpr int BLOCK = SBLOCK;
constexpr int OPL = 4;
constexpr uint64_t CHUNK = (uint64_t)BLOCK * OPL;
constexpr uint32_t LB = 1024;   // LDS births per chunk
constexpr uint32_t LK = 2048;   // LDS kills per chunk
constexpr uint32_t SCAP = 2048; // survivors sorted in LDS by k_big_finish
constexpr uint32_t HEMPTY = 0xFFFFFFFFu;

struct BigRead {
  uint64_t r, off0, off1;
  uint64_t chunk0;  // first flattened chunk
  uint64_t rec0;    // first record slot (births and kills each have cap slots)
  uint64_t cap;     // record capacity (power of two: the global sort pads to it)
  uint64_t h0;      // first hash slot
  uint64_t hmask;   // hash slots - 1
  uint64_t bm0;     // grouped mode: first word of the born | killed group bitmaps
  uint64_t gchunk0; // k_big_run's reads: first chunk in its chunk space
  uint32_t G;       // grouped mode: the key's groups (chunked token-group view)
  uint32_t grouped;
};

struct BigAcc {
  uint32_t count, flags, pres, nbirth, nkill, pad0;
  unsigned long long min_excl;
  unsigned long long mx[AM_MAX_DC];
};

struct BigSlots {  // bounded counter: ns slots per big read (P: D*D, D: D)
  uint64_t *lo;
  int64_t *hi;
  uint32_t *pres;
  uint32_t ns;
};

struct BigRec {
  uint64_t *ba, *bb;  // births: output pair
  int32_t *bp;        // birth position (-1 = base snapshot)
  uint32_t *bs;       // birth: index in the effect's token list (base: in the base list)
  uint64_t *ot;       // finish: AW survivor tokens (global-scratch sort)
  int32_t *oi;        // finish: AW survivor index (global-scratch sort payload)
  uint32_t *bm;       // grouped mode: per read born [gw] | killed [gw] bitmaps
  uint32_t *ibm;      // grouped mode: per chunk inclusion bits (32 words)
  uint8_t *dead;
  uint64_t *ka, *kb;  // exported kills: kill key
  int32_t *kp;
  uint32_t *H;        // hash slots: birth record index (relative to rec0)
};

__device__ __forceinline__ uint64_t next_pow2(uint64_t x) {
  uint64_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

__device__ __forceinline__ uint64_t key_hash(uint64_t a, uint64_t b) {
  uint64_t h = a * 0x9E3779B97F4A7C15ull ^ (b + 0x632BE59BD9B4E019ull) * 0xC2B2AE3D27D4EB4Full;
  h ^= h >> 29;
  h *= 0xBF58476D1CE4E5B9ull;
  return h ^ (h >> 32);
}

// last index i with v[i].field <= x (v sorted ascending, v[0].field == 0)
template <typename F>
__device__ __forceinline__ uint32_t find_read(const BigRead *br, uint32_t nbig, uint64_t x, F field) {
  uint32_t lo = 0, hi = nbig;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (field(br[mid]) <= x) lo = mid;
    else hi = mid;
  }
  return lo;
}

// ---- prep: per big read sizes (sz[0..2][b] = chunks, record cap, hash slots) ----
template <int TYPE>
__global__ void k_big_prep(am_op_log L, am_read_batch B, const uint32_t *list, const uint32_t *nbig_p, BigRead *br,
                           BigAcc *acc, uint64_t *sz, BigSlots SL) {
  const uint32_t nbig = *nbig_p;
  for (uint32_t b = blockIdx.x * blockDim.x + threadIdx.x; b < nbig; b += gridDim.x * blockDim.x) {
    const uint64_t r = list[b];
    const uint64_t key = B.key[r];
    const uint64_t off0 = L.key_off[key], off1 = am_kend(L, key);
    const uint64_t W = L.var_off ? L.var_off[off1] - L.var_off[off0] : 0;
    const uint64_t nbase = B.base.set_off ? B.base.set_len[r] : 0;
    const uint64_t t0 = off0 & ~(uint64_t)(OPL - 1);
    const uint64_t nch = off1 > t0 ? (off1 - t0 + CHUNK - 1) / CHUNK : 1;
    // births: AW <= add tokens <= W, MV <= ops; kills <= W; + base pairs
    // grouped mode: an MV key with the chunked token-group view and no base pairs
    const uint32_t ng = (TYPE == AM_MVREG && L.key_ngrp && L.rec_g) ? L.key_ngrp[key] : AM_NGRP_NONE;
    const bool grouped = am_ngrp_big(ng) && nbase == 0;
    const uint32_t G = grouped ? am_ngrp_count(ng) : 0u;
    const uint64_t cap =
        (TYPE == AM_BCOUNTER || grouped) ? 1 : next_pow2((W > off1 - off0 ? W : off1 - off0) + nbase + 1);
    BigRead x;
    x.r = r, x.off0 = off0, x.off1 = off1, x.chunk0 = 0, x.rec0 = 0, x.cap = cap, x.h0 = 0, x.hmask = 2 * cap - 1;
    x.bm0 = 0, x.G = G, x.grouped = grouped ? 1u : 0u;
    br[b] = x;
    const bool run = grouped || TYPE == AM_BCOUNTER;  // k_big_run's reads (its own chunk space)
    sz[b] = run ? 0 : nch;
    sz[(uint64_t)nbig + b] = cap;
    sz[2 * (uint64_t)nbig + b] = grouped ? 2 * (uint64_t)((G + 31) / 32) : 0;
    sz[3 * (uint64_t)nbig + b] = run ? nch : 0;
    BigAcc a;
    a.count = a.flags = a.pres = a.nbirth = a.nkill = a.pad0 = 0;
    a.min_excl = NONE;
    for (int d = 0; d < AM_MAX_DC; ++d) a.mx[d] = 0;
    acc[b] = a;
  }
  if (TYPE == AM_BCOUNTER) {  // slots start from the base snapshot's orddicts: one thread per slot
    const uint32_t nd = L.n_dc, np = nd * nd;
    const uint64_t nq = (uint64_t)nbig * SL.ns;
    for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nq; q += (uint64_t)gridDim.x * blockDim.x) {
      const uint32_t b = (uint32_t)(q / SL.ns), i = (uint32_t)(q % SL.ns);
      uint32_t bp = 0;
      const int64_t bv = bc_base(B, list[b], np, nd, i, bp);
      SL.lo[q] = (uint64_t)bv;
      SL.hi[q] = bv < 0 ? -1 : 0;
      SL.pres[q] = bp;
    }
  }
}

// one workgroup of 1024: exclusive scans of chunks, caps, bitmap words and grouped-mode
// chunks; totals[0..3]
__global__ void __launch_bounds__(1024) k_big_offsets(const uint32_t *nbig_p, BigRead *br, const uint64_t *sz,
                                                      uint64_t *totals) {
  __shared__ uint64_t part[1024];
  const uint32_t nbig = *nbig_p, tid = threadIdx.x;
  const uint32_t per = (nbig + 1023) / 1024;
  const uint32_t b0 = tid * per < nbig ? tid * per : nbig, b1 = b0 + per < nbig ? b0 + per : nbig;
  for (int f = 0; f < 4; ++f) {
    const uint64_t *v = sz + (uint64_t)f * nbig;
    uint64_t s = 0;
    for (uint32_t b = b0; b < b1; ++b) s += v[b];
    part[tid] = s;
    __syncthreads();
    for (uint32_t o = 1; o < 1024; o <<= 1) {
      const uint64_t w = tid >= o ? part[tid - o] : 0;
      __syncthreads();
      part[tid] += w;
      __syncthreads();
    }
    uint64_t run = part[tid] - s;
    for (uint32_t b = b0; b < b1; ++b) {
      if (f == 0) br[b].chunk0 = run;
      else if (f == 1) br[b].rec0 = run, br[b].h0 = 2 * run;
      else if (f == 2) br[b].bm0 = run;
      else br[b].gchunk0 = run;
      run += v[b];
    }
    if (tid == 1023) totals[f] = part[1023];
    __syncthreads();
  }
}

// ---- chunk: inclusion + local resolution + export ----
struct ChunkSmem {
  uint64_t lb_a[LB], lb_b[LB];
  int32_t lb_p[LB];
  uint32_t lb_s[LB];
  uint64_t lk_a[LK], lk_b[LK];
  int32_t lk_p[LK];
  uint32_t ctr[8];  // [0] kills [1] births
  uint64_t red[4];
};

// MV register chunks keep their kills in an LDS hash on the token (the MV kill key) holding
// the latest kill position, instead of a list bitonic-sorted per chunk: insert = one 64-bit
// LDS CAS + atomicMax, a birth's lookup = a few probes.  A kill that finds no slot goes
// straight to the global records (resolved by the global pass, like an LDS overflow).
constexpr uint64_t HKEY_EMPTY = ~0ull;
constexpr uint32_t HPROBES = 64;
__device__ __forceinline__ uint32_t tok_slot(uint64_t t) { return (uint32_t)(key_hash(t, 0) & (LK - 1)); }

struct ChunkSink {
  ChunkSmem *s;
  BigRec G;
  BigAcc *acc;
  uint64_t rec0;
  bool mvhash;  // MV register: kills into the LDS token hash
  __device__ void gbirth(uint64_t a, uint64_t b, int32_t pos, uint32_t sub) {
    const uint64_t i = rec0 + atomicAdd(&acc->nbirth, 1u);
    G.ba[i] = a, G.bb[i] = b, G.bp[i] = pos, G.bs[i] = sub;
  }
  template <int TYPE>
  __device__ void gkill(uint64_t tok, uint64_t e, int32_t pos) {
    const uint64_t i = rec0 + atomicAdd(&acc->nkill, 1u);
    G.ka[i] = tok, G.kb[i] = TYPE == AM_AWSET ? e : 0ull, G.kp[i] = pos;
  }
  __device__ void births(uint64_t e, const uint64_t *tok, uint32_t n, int32_t pos) {
    for (uint32_t i = 0; i < n; ++i) birth_s(e, tok[i], pos, i);
  }
  __device__ void birth(uint64_t a, uint64_t b, int32_t pos) { birth_s(a, b, pos, 0); }
  __device__ void birth_s(uint64_t a, uint64_t b, int32_t pos, uint32_t sub) {
    const uint32_t bi = atomicAdd(&s->ctr[1], 1u);
    if (bi < LB) s->lb_a[bi] = a, s->lb_b[bi] = b, s->lb_p[bi] = pos, s->lb_s[bi] = sub;
    else gbirth(a, b, pos, sub);  // LDS full: unresolved, straight to the global records
  }
  __device__ bool hash_kill(uint64_t t, int32_t pos) {
    if (t == HKEY_EMPTY) return false;
    const uint32_t h = tok_slot(t);
    for (uint32_t pr = 0; pr < HPROBES; ++pr) {
      const uint32_t sl = (h + pr) & (LK - 1);
      const unsigned long long old =
          atomicCAS((unsigned long long *)&s->lk_a[sl], (unsigned long long)HKEY_EMPTY, (unsigned long long)t);
      if (old == HKEY_EMPTY || old == t) {
        atomicMax(&s->lk_p[sl], pos);
        return true;
      }
    }
    return false;
  }
  __device__ void kills(const uint64_t *tok, uint32_t n, uint64_t e, int32_t pos) {
    for (uint32_t i = 0; i < n; ++i) {
      if (mvhash) {
        if (!hash_kill(tok[i], pos)) gkill<AM_AWSET>(tok[i], e, pos);  // e is 0 for MV kills
        continue;
      }
      const uint32_t ki = atomicAdd(&s->ctr[0], 1u);
      if (ki < LK) s->lk_a[ki] = tok[i], s->lk_b[ki] = e, s->lk_p[ki] = pos;
      else gkill<AM_AWSET>(tok[i], e, pos);  // e is 0 for MV kills already
    }
  }
};

// ---- grouped mode (chunked token-group view, am_grpbig.hip): a group survives iff its birth
//      is included and no kill of it is (effective kills follow the birth), so births and kills
//      are sets.  A chunk collects its included births and kills in two LDS hash sets and
//      exports only what it cannot settle itself: a group born and killed within the chunk is
//      dead (one birth per group), so neither bit leaves; the rest are ORed into the read's
//      born / killed bitmaps.  An MV override chain leaves about one bit of each per chunk. ----
constexpr uint32_t GH = LK;          // slots per hash set (two sets in ChunkSmem::lk_a)
constexpr uint32_t GH_EMPTY = 0xFFFFFFFFu;
__device__ __forceinline__ uint32_t gslot(uint32_t g) { return (g * 0x9E3779B1u) >> 21; }  // 11 bits
static_assert(GH == 2048, "gslot yields 11 bits");
__device__ __forceinline__ bool gset_insert(uint32_t *h, uint32_t g) {
  const uint32_t s0 = gslot(g);
  for (uint32_t pr = 0; pr < 32; ++pr) {
    const uint32_t sl = (s0 + pr) & (GH - 1);
    const uint32_t old = atomicCAS(&h[sl], GH_EMPTY, g);
    if (old == GH_EMPTY || old == g) return true;
  }
  return false;
}
__device__ __forceinline__ bool gset_has(const uint32_t *h, uint32_t g) {
  const uint32_t s0 = gslot(g);
  for (uint32_t pr = 0; pr < 32; ++pr) {
    const uint32_t x = h[(s0 + pr) & (GH - 1)];
    if (x == g) return true;
    if (x == GH_EMPTY) return false;
  }
  return false;
}
// the records of chunk ops [lo, hi) (incl: their inclusion bits from lo); hs = 2 * GH u32 of
// LDS at GH_EMPTY; bm = the read's born [gw] | killed [gw] words
__device__ void grouped_records(const am_op_log &L, uint64_t key, const BigRead &R0, uint64_t lo, uint64_t hi,
                                const uint32_t *incl, uint32_t *hs, uint32_t *bm, uint32_t tid) {
  uint32_t *hb = hs, *hk = hs + GH;
  const uint32_t gw = (R0.G + 31) / 32;
  const uint64_t rk0 = L.rec_key_off[key];
  const uint64_t ka = (lo > R0.off0 ? lo : R0.off0) - R0.off0, kb = hi - R0.off0;  // key op range
  for (uint64_t hc = ka / AM_BIG_CHUNK; hc <= (kb - 1) / AM_BIG_CHUNK; ++hc) {
    const uint64_t a0 = rk0 + L.rec_g[rk0 + hc], a1 = rk0 + L.rec_g[rk0 + hc + 1];
    for (uint64_t q = a0 + tid; q < a1; q += BLOCK) {
      const uint32_t x = L.rec_g[q];
      if (x == 0xFFFFFFFFu) continue;  // an ineffective kill
      const uint64_t op = hc * AM_BIG_CHUNK + AM_BREC_OP(x);
      if (op < ka || op >= kb) continue;
      const uint32_t bit = (uint32_t)(op + R0.off0 - lo);
      if (!((incl[bit >> 5] >> (bit & 31)) & 1u)) continue;
      const uint32_t g = AM_BREC_GRP(x);
      const bool kill = (x & AM_BREC_KILL) != 0;
      if (!gset_insert(kill ? hk : hb, g)) atomicOr(bm + (kill ? gw : 0u) + (g >> 5), 1u << (g & 31));
    }
  }
  __syncthreads();
  for (uint32_t sl = tid; sl < GH; sl += BLOCK) {
    const uint32_t b = hb[sl], k = hk[sl];
    if (b != GH_EMPTY && !gset_has(hk, b)) atomicOr(bm + (b >> 5), 1u << (b & 31));
    if (k != GH_EMPTY && !gset_has(hb, k)) atomicOr(bm + gw + (k >> 5), 1u << (k & 31));
  }
}

template <int DMAX, int TYPE, bool PACKED>
__global__ void __launch_bounds__(BLOCK) k_big_chunk(am_op_log L, am_read_batch B, const uint32_t *nbig_p,
                                                     const BigRead *br, BigAcc *accs, BigRec G, BigSlots SL,
                                                     uint64_t n_chunks) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  ChunkSmem &s = *(ChunkSmem *)smem_raw;
  const uint32_t tid = threadIdx.x;
  const uint32_t nbig = uniform_u32(*nbig_p);
  const uint64_t n = B.n_reads;
  const uint32_t nd = L.n_dc;
  const uint64_t stride = L.snap_stride ? L.snap_stride : L.n_ops;

  for (uint64_t x = blockIdx.x; x < n_chunks; x += gridDim.x) {
    const uint32_t b = find_read(br, nbig, x, [](const BigRead &v) { return v.chunk0; });
    const BigRead R0 = br[b];
    const uint64_t r = R0.r;
    BigAcc *acc = accs + b;
    const uint64_t t0 = R0.off0 & ~(uint64_t)(OPL - 1);
    const uint64_t c = x - R0.chunk0;
    const uint64_t lo = t0 + c * CHUNK, hi = lo + CHUNK < R0.off1 ? lo + CHUNK : R0.off1;

    ReadU<DMAX> u;
    u.allmask = nd >= 32 ? 0xFFFFFFFFu : ((1u << nd) - 1u);
    const uint64_t rstride = B.per_read_clock ? n : 1, ridx = B.per_read_clock ? r : 0;
    u.spres = uniform_u32(B.read_pres[ridx]) & u.allmask;
    u.base_ignore = !B.base_ignore || B.base_ignore[r];
    u.cpres = u.base_ignore ? 0u : (uniform_u32(B.base_pres[r]) & u.allmask);
#pragma unroll
    for (int d = 0; d < DMAX; ++d) {
      u.S[d] = (d < (int)nd && ((u.spres >> d) & 1u)) ? uniform_u64(B.read_vc[(uint64_t)d * rstride + ridx]) : 0;
      u.C0[d] = (d < (int)nd && ((u.cpres >> d) & 1u)) ? uniform_u64(B.base_vc[(uint64_t)d * n + r]) : 0;
    }
    u.has_txid = B.txid && (!B.txid_valid || B.txid_valid[r]) && L.op_txid;
    u.txid = u.has_txid ? uniform_u64(B.txid[r]) : 0;

    if (tid < 8) s.ctr[tid] = 0;
    constexpr bool MVH = TYPE == AM_MVREG;
    if (MVH)
      for (uint32_t i = tid; i < LK; i += BLOCK) s.lk_a[i] = HKEY_EMPTY, s.lk_p[i] = (int32_t)0x80000000;
    ChunkSink sink{&s, G, acc, R0.rec0, MVH};
    uint64_t *slo = s.lk_a;  // bounded counter: LDS slot sums of this chunk
    int64_t *shi = (int64_t *)s.lk_b;
    uint32_t *spres = (uint32_t *)s.lk_p;
    if (TYPE == AM_BCOUNTER)
      for (uint32_t i = tid; i < SL.ns; i += BLOCK) slo[i] = 0, shi[i] = 0, spres[i] = 0;
    __syncthreads();
    if (TYPE != AM_BCOUNTER && c == 0 && B.base.set_off) {  // base snapshot pairs: births at -1 (no later kill in
      const uint64_t bo = B.base.set_off[r];  // this chunk can be ruled out, so global)
      const uint32_t bl = B.base.set_len[r];
      for (uint32_t i = tid; i < bl; i += BLOCK) sink.gbirth(B.base.set_a[bo + i], B.base.set_b[bo + i], -1, i);
    }

    Acc<DMAX> a;
    a.reset();
    AccP<DMAX> ap;
    ap.reset();
    PkRead<DMAX> pk;
    if (PACKED) pk_setup(u, nd, uniform_u64(L.key_tbase[uniform_u64(B.key[r])]), pk);
    const uint64_t g = lo + (uint64_t)tid * OPL;
    if (g < hi) {
      const uint32_t meta4 = *(const uint32_t *)(L.op_meta + g);
      uint32_t ib = 0;
      if constexpr (PACKED) {
        ib = incl4<DMAX, true>(L, nd, stride, u, pk, g, R0.off0, hi, ap, a);
      } else {
        const u64x2 c01 = *(const u64x2 *)(L.commit_time + g), c23 = *(const u64x2 *)(L.commit_time + g + 2);
        const uint64_t ct[OPL] = {c01.x, c01.y, c23.x, c23.y};
        uint64_t sv[OPL][DMAX];
#pragma unroll
        for (int d = 0; d < DMAX; ++d) {
          if (d < (int)nd) {
            const uint64_t *col = L.snap_vc + (uint64_t)d * stride + g;
            const u64x2 s01 = *(const u64x2 *)col, s23 = *(const u64x2 *)(col + 2);
            sv[0][d] = s01.x, sv[1][d] = s01.y, sv[2][d] = s23.x, sv[3][d] = s23.y;
          } else {
            sv[0][d] = sv[1][d] = sv[2][d] = sv[3][d] = 0;
          }
        }
        uint32_t sp[OPL] = {u.allmask, u.allmask, u.allmask, u.allmask};
        if (L.snap_pres) {
          const u32x4 q = *(const u32x4 *)(L.snap_pres + g);
          sp[0] = q.x, sp[1] = q.y, sp[2] = q.z, sp[3] = q.w;
        }
#pragma unroll
        for (int k = 0; k < OPL; ++k) {
          const uint64_t p = g + k;
          if (p < R0.off0 || p >= hi) continue;
          const bool txm = u.has_txid && L.op_txid[p] == u.txid;
          if (eval_op<DMAX, true>(u, (meta4 >> (8 * k)) & 0xFFu, ct[k], sv[k], sp[k], txm, p, a)) ib |= 1u << k;
        }
      }
#pragma unroll
      for (int k = 0; k < OPL; ++k) {
        if (!((ib >> k) & 1u)) continue;
        const uint64_t p = g + k;
        const uint32_t meta = (meta4 >> (8 * k)) & 0xFFu;
        if (meta & AM_META_BAD) continue;  // reported through FLAG_BAD
        if (TYPE == AM_BCOUNTER) {
          uint32_t slot;
          int64_t v;
          if (!bc_slot(L, p, meta, nd, slot, v)) {
            a.flags |= FLAG_BAD;
            continue;
          }
          acc128_atomic(&slo[slot], &shi[slot], v < 0 ? -1 : 0, (uint64_t)v);
          atomicOr(&spres[slot], 1u);
        } else if (!set_effects<TYPE>(L, p, meta, (int32_t)(p - R0.off0), sink)) {
          a.flags |= FLAG_BAD;
        }
      }
    }
    if (PACKED) pk_fold(ap, pk.K, u.allmask, a);
    __syncthreads();

    // ---- scalar partials -> the read's accumulators ----
    const uint32_t count = (uint32_t)block_red_u64(s.red, wave_sum_u32(a.count), 0);
    const uint32_t flags = (uint32_t)block_red_u64(s.red, wave_or_u32(a.flags), 1);
    const uint32_t pres = (uint32_t)block_red_u64(s.red, wave_or_u32(a.pres), 1);
    const uint64_t min_excl = block_red_u64(s.red, wave_min_u64(a.min_excl), 3);
    uint64_t mx[DMAX];
#pragma unroll
    for (int d = 0; d < DMAX; ++d) mx[d] = d < (int)nd ? block_red_u64(s.red, wave_max_u64(a.mx[d]), 2) : 0;
    if (tid == 0) {
      if (count) atomicAdd(&acc->count, count);
      if (flags) atomicOr(&acc->flags, flags);
      if (pres) atomicOr(&acc->pres, pres);
      if (min_excl != NONE) atomicMin(&acc->min_excl, (unsigned long long)min_excl);
      for (int d = 0; d < DMAX; ++d)
        if (d < (int)nd && mx[d]) atomicMax(&acc->mx[d], (unsigned long long)mx[d]);
    }

    if (TYPE == AM_BCOUNTER) {  // flush the chunk's slot sums into the read's global slots
      for (uint32_t i = tid; i < SL.ns; i += BLOCK) {
        const uint64_t q = (uint64_t)b * SL.ns + i;
        if (slo[i] || shi[i]) acc128_atomic(&SL.lo[q], &SL.hi[q], shi[i], slo[i]);
        if (spres[i]) atomicOr(&SL.pres[q], 1u);
      }
      __syncthreads();
      continue;
    }
    // ---- local resolution, then export ----
    if constexpr (MVH) {  // kills are in the LDS token hash
      const uint32_t nb = s.ctr[1] < LB ? s.ctr[1] : LB;
      for (uint32_t i = tid; i < nb; i += BLOCK) {
        const uint64_t t = s.lb_b[i];  // MV kill key of the birth (value, token): its token
        bool dead = false;
        if (t != HKEY_EMPTY) {
          const uint32_t h = tok_slot(t);
          for (uint32_t pr = 0; pr < HPROBES; ++pr) {
            const uint32_t sl = (h + pr) & (LK - 1);
            const uint64_t k = s.lk_a[sl];
            if (k == t) {
              dead = s.lk_p[sl] > s.lb_p[i];
              break;
            }
            if (k == HKEY_EMPTY) break;
          }
        }
        if (!dead) sink.gbirth(s.lb_a[i], s.lb_b[i], s.lb_p[i], s.lb_s[i]);
      }
      for (uint32_t sl = tid; sl < LK; sl += BLOCK)  // the latest kill of each token
        if (s.lk_a[sl] != HKEY_EMPTY) sink.gkill<AM_AWSET>(s.lk_a[sl], 0ull, s.lk_p[sl]);
      __syncthreads();
      continue;
    }
    const uint32_t nk = s.ctr[0] < LK ? s.ctr[0] : LK;
    const uint32_t nb = s.ctr[1] < LB ? s.ctr[1] : LB;
    block_sort(s.lk_a, s.lk_b, s.lk_p, nk, LK);  // by (kill key, pos)
    for (uint32_t i = tid; i < nb; i += BLOCK) {
      uint64_t qa, qb;
      birth_kill_key<TYPE>(s.lb_a[i], s.lb_b[i], qa, qb);
      uint32_t l = 0, h = nk;  // upper bound of (qa, qb, +inf)
      while (l < h) {
        const uint32_t mid = (l + h) >> 1;
        const bool le = s.lk_a[mid] < qa || (s.lk_a[mid] == qa && s.lk_b[mid] <= qb);
        if (le) l = mid + 1;
        else h = mid;
      }
      const bool dead = l > 0 && s.lk_a[l - 1] == qa && s.lk_b[l - 1] == qb && s.lk_p[l - 1] > s.lb_p[i];
      if (!dead) sink.gbirth(s.lb_a[i], s.lb_b[i], s.lb_p[i], s.lb_s[i]);
    }
    for (uint32_t i = tid; i < nk; i += BLOCK) {  // the latest kill of each key
      if (i + 1 == nk || s.lk_a[i + 1] != s.lk_a[i] || s.lk_b[i + 1] != s.lk_b[i])
        sink.gkill<AM_AWSET>(s.lk_a[i], s.lk_b[i], s.lk_p[i]);
    }
    __syncthreads();
  }
}

// ---- LEAN evaluation (packed view, the batch clock: no bases / TxIds / op presence): the clock
//      is read once per kernel and the chunk loops test the packed entries only; an escaped op
//      is evaluated from the full columns one DC at a time (lane d's vS holds the clock's entry
//      d) with its LastOpCt maxima into an LDS array -- the loops hold no D-wide u64 arrays
//      (D = 16: k_big_gincl 227 -> 155 VGPRs).  eval_op<DMAX, false> semantics. ----
template <int DMAX>
__device__ __forceinline__ void lean_clock(const am_read_batch &B, uint32_t nd, uint32_t lane, ReadU<DMAX> &u,
                                           uint64_t &vS) {
  u.allmask = nd >= 32 ? 0xFFFFFFFFu : ((1u << nd) - 1u);
  u.spres = uniform_u32(B.read_pres[0]) & u.allmask;
  u.base_ignore = true, u.cpres = 0, u.has_txid = false, u.txid = 0;
  vS = 0;
#pragma unroll
  for (int d = 0; d < DMAX; ++d) {
    u.S[d] = (d < (int)nd && ((u.spres >> d) & 1u)) ? uniform_u64(B.read_vc[d]) : 0;
    u.C0[d] = 0;
    vS = (uint32_t)d == lane ? u.S[d] : vS;
  }
}
// the 4 ops [g, g + 4) of a read inside [lo, hi): inclusion bits; packed partials in ap, the
// escaped ops' count / flags / min in a and their maxima in emx
template <int DMAX>
__device__ __forceinline__ uint32_t lean_incl4(const am_op_log &L, uint32_t nd, uint64_t stride, const ReadU<DMAX> &u,
                                               const PkRead<DMAX> &pk, const LagRead<DMAX> &lr, uint64_t vS,
                                               uint64_t g, uint64_t lo, uint64_t hi, AccP<DMAX> &ap, Acc<DMAX> &a,
                                               unsigned long long *emx) {
  const uint64_t tx[4] = {0, 0, 0, 0};
  bool esc = false;
  uint32_t ib;
  if (lr.on) {  // the lag view: 4 + 2 D bytes per op
    const u32x4 cq = *(const u32x4 *)(L.lag_ct + g);
    const uint32_t c[4] = {cq.x, cq.y, cq.z, cq.w};
    uint32_t lw[DMAX][2];
#pragma unroll
    for (int d = 0; d < DMAX; ++d) {
      const uint2 v = d < (int)nd ? *(const uint2 *)(L.lag + (uint64_t)d * stride + g) : uint2{0, 0};
      lw[d][0] = v.x, lw[d][1] = v.y;
    }
    ib = pk_tile_lag<DMAX, 4, false>(u, pk, lr, c, lw, tx, g, lo, hi, ap, esc);
  } else {
    uint32_t xs[4][DMAX];
#pragma unroll
    for (int d = 0; d < DMAX; ++d) {
      u32x4 q = {0, 0, 0, 0};
      if (d < (int)nd) q = *(const u32x4 *)(L.pk_vc + (uint64_t)d * stride + g);
      xs[0][d] = q.x, xs[1][d] = q.y, xs[2][d] = q.z, xs[3][d] = q.w;
    }
    ib = pk_tile<DMAX, 4, false>(u, pk, xs, tx, g, lo, hi, ap, esc);
  }
  if (!esc) return ib;
  const uint32_t *escv = lr.on ? L.lag_ct : L.pk_vc;
#pragma unroll 1
  for (int k = 0; k < 4; ++k) {  // rare
    const uint64_t p = g + k;
    if (p < lo || p >= hi || escv[p] != AM_PK_ESC) continue;
    const uint64_t *w = esc_row(L, stride, p);  // its escape row, or the columns
    const uint32_t meta = w ? (uint32_t)w[1] : L.op_meta[p], dc = meta & 31u;
    const uint64_t ct = w ? w[0] : L.commit_time[p];
    bool in = true;
    for (uint32_t d = 0; d < nd; ++d) {
      if (!((u.spres >> d) & 1u)) {  // logger:error("Could not find DC in SS"); excluded
        in = false;
        a.flags |= AM_FLAG_MISSING_DC_LOGGED;
        continue;
      }
      in &= (d == dc ? ct : (w ? w[2 + d] : L.snap_vc[(uint64_t)d * stride + p])) <= lane_u64(vS, d);
    }
    if (!in) {
      a.min_excl = p < a.min_excl ? p : a.min_excl;
      continue;
    }
    for (uint32_t d = 0; d < nd; ++d)
      atomicMax(&emx[d], (unsigned long long)(d == dc ? ct : (w ? w[2 + d] : L.snap_vc[(uint64_t)d * stride + p])));
    a.pres |= u.allmask;
    a.count += 1;
    if (meta & AM_META_BAD) a.flags |= FLAG_BAD;
    ib |= 1u << k;
  }
  return ib;
}
// a wave's LastOpCt maxima of the read (LEAN: from the packed partials; else from a) and the
// packed partials folded into a's counts
template <int DMAX, bool PACKED, bool LEAN>
__device__ __forceinline__ void wave_partials(AccP<DMAX> &ap, const PkRead<DMAX> &pk, const ReadU<DMAX> &u,
                                              uint32_t nd, Acc<DMAX> &a, uint64_t (&mx)[DMAX]) {
  if constexpr (LEAN) {
#pragma unroll
    for (int d = 0; d < DMAX; ++d) mx[d] = d < (int)nd ? wave_max_u64(ap.count ? pk.K + ap.mx[d] : 0) : 0;
    a.count += ap.count, a.flags |= ap.flags;
    if (ap.count) a.pres |= u.allmask;
    a.min_excl = umin64(a.min_excl, ap.min_excl);
  } else {
    if (PACKED) pk_fold(ap, pk.K, u.allmask, a);
#pragma unroll
    for (int d = 0; d < DMAX; ++d) mx[d] = d < (int)nd ? wave_max_u64(a.mx[d]) : 0;
  }
}

// ---- runs of chunks: grouped-mode MV reads and bounded-counter reads.  A workgroup takes a
//      contiguous run of 1024-op chunks, so a read's partials stay on the workgroup across its
//      chunks -- the scalar partials in registers, the bounded counter's slot sums in LDS --
//      and reach the read's accumulators once per read and workgroup (k_big_chunk reduces and
//      flushes every chunk).  LDS holds only what the type needs: MV the two hash sets, the
//      bounded counter its slot sums (k_big_chunk's 64 KB allow two workgroups per CU). ----
#ifndef AM_BIGRUN_LAG
#define AM_BIGRUN_LAG 0  // the bounded-counter runs keep the packed view: the lag branch costs them
#endif                   // an occupancy step (D = 16: 163 -> 173 VGPRs, 3 -> 2 waves)
template <int DMAX, int TYPE, bool PACKED, bool LEAN = false>
__global__ void __launch_bounds__(BLOCK) k_big_run(am_op_log L, am_read_batch B, const uint32_t *nbig_p,
                                                   const BigRead *br, BigAcc *accs, uint32_t *bm, BigSlots SL,
                                                   uint64_t n_gch) {
  constexpr uint32_t NS = (uint32_t)(DMAX * DMAX + DMAX);
  constexpr size_t HB = TYPE == AM_MVREG ? 2 * GH * 4 : (size_t)NS * 20;
  __shared__ __attribute__((aligned(16))) unsigned char lds[HB];
  uint32_t *hs = reinterpret_cast<uint32_t *>(lds);  // MV: hash sets
  uint64_t *slo = reinterpret_cast<uint64_t *>(lds);  // bounded counter: 128-bit slot sums + presence
  int64_t *shi = reinterpret_cast<int64_t *>(lds + (size_t)NS * 8);
  uint32_t *spres = reinterpret_cast<uint32_t *>(lds + (size_t)NS * 16);
  __shared__ uint32_t incl[CHUNK / 32];
  __shared__ uint64_t red[BLOCK / WAVE][DMAX + 4];
  __shared__ unsigned long long emx[DMAX];  // LEAN: the read's escaped ops' LastOpCt maxima
  const uint32_t tid = threadIdx.x, lane = tid & (WAVE - 1), wv = tid / WAVE;
  const uint32_t nbig = uniform_u32(*nbig_p);
  const uint64_t n = B.n_reads;
  const uint32_t nd = L.n_dc;
  const uint64_t stride = L.snap_stride ? L.snap_stride : L.n_ops;
  const uint64_t per = (n_gch + gridDim.x - 1) / gridDim.x;
  const uint64_t x0 = (uint64_t)blockIdx.x * per < n_gch ? (uint64_t)blockIdx.x * per : n_gch;
  const uint64_t x1 = x0 + per < n_gch ? x0 + per : n_gch;
  uint32_t cur = 0xFFFFFFFFu;
  BigRead R0{};
  ReadU<DMAX> u;
  PkRead<DMAX> pk;
  AccP<DMAX> ap;
  Acc<DMAX> a;
  // the read's partials -> its accumulators (one LDS round over the waves)
  uint64_t vS = 0;  // LEAN: lane d holds the clock's entry d
  LagRead<DMAX> lr;  // LEAN: the read's lag bases (the lag view, when the store has one)
  lr.on = false;
  auto flush = [&]() {
    uint64_t mx[DMAX];
    wave_partials<DMAX, PACKED, LEAN>(ap, pk, u, nd, a, mx);
    const uint32_t cnt = wave_sum_u32(a.count), fl = wave_or_u32(a.flags), pr = wave_or_u32(a.pres);
    const uint64_t mn = wave_min_u64(a.min_excl);
    if (lane == 0) {
      red[wv][0] = cnt, red[wv][1] = fl, red[wv][2] = pr, red[wv][3] = mn;
#pragma unroll
      for (int d = 0; d < DMAX; ++d) red[wv][4 + d] = mx[d];
    }
    __syncthreads();
    if (tid < 4 + (uint32_t)DMAX) {
      uint64_t v = red[0][tid];
      for (uint32_t w = 1; w < BLOCK / WAVE; ++w) {
        const uint64_t y = red[w][tid];
        v = tid == 0 ? v + y : (tid <= 2 ? (v | y) : tid == 3 ? (v < y ? v : y) : (v > y ? v : y));
      }
      if (LEAN && tid >= 4) v = v > emx[tid - 4] ? v : emx[tid - 4];
      BigAcc *acc = accs + cur;
      if (tid == 0 && v) atomicAdd(&acc->count, (uint32_t)v);
      if (tid == 1 && v) atomicOr(&acc->flags, (uint32_t)v);
      if (tid == 2 && v) atomicOr(&acc->pres, (uint32_t)v);
      if (tid == 3 && v != NONE) atomicMin(&acc->min_excl, (unsigned long long)v);
      if (tid >= 4 && tid - 4 < nd && v) atomicMax(&acc->mx[tid - 4], (unsigned long long)v);
    }
    if (TYPE == AM_BCOUNTER) {  // the slot sums -> the read's global slots, then cleared
      for (uint32_t i = tid; i < SL.ns; i += BLOCK) {
        const uint64_t q = (uint64_t)cur * SL.ns + i;
        if (slo[i] || shi[i]) acc128_atomic(&SL.lo[q], &SL.hi[q], shi[i], slo[i]);
        if (spres[i]) atomicOr(&SL.pres[q], 1u);
        slo[i] = 0, shi[i] = 0, spres[i] = 0;
      }
    }
    __syncthreads();
  };
  if (TYPE == AM_BCOUNTER) {
    for (uint32_t i = tid; i < SL.ns; i += BLOCK) slo[i] = 0, shi[i] = 0, spres[i] = 0;
    __syncthreads();
  }
  if constexpr (LEAN) lean_clock<DMAX>(B, nd, lane, u, vS);
  for (uint64_t x = x0; x < x1; ++x) {
    // a workgroup's run mostly stays in one read: search the read list (a chain of dependent
    // loads) only when x leaves the current read's chunks
    const bool same = cur != 0xFFFFFFFFu && x < R0.gchunk0 + ((R0.off1 - (R0.off0 & ~(uint64_t)(OPL - 1)) + CHUNK - 1) / CHUNK);
    const uint32_t b = same ? cur : find_read(br, nbig, x, [](const BigRead &v) { return v.gchunk0; });
    if (b != cur && LEAN) {
      if (cur != 0xFFFFFFFFu) flush();
      cur = b;
      R0 = br[b];
      if (tid < DMAX) emx[tid] = 0;
      __syncthreads();
      const uint64_t key = uniform_u64(B.key[R0.r]);
      pk_setup(u, nd, uniform_u64(L.key_tbase[key]), pk);
      lag_setup(L, nd, key, AM_BIGRUN_LAG && L.lag_ct != nullptr, lr);
      ap.reset();
      a.reset();
    } else if (b != cur) {
      if (cur != 0xFFFFFFFFu) flush();
      cur = b;
      R0 = br[b];
      const uint64_t r = R0.r;
      u.allmask = nd >= 32 ? 0xFFFFFFFFu : ((1u << nd) - 1u);
      const uint64_t rstride = B.per_read_clock ? n : 1, ridx = B.per_read_clock ? r : 0;
      u.spres = uniform_u32(B.read_pres[ridx]) & u.allmask;
      u.base_ignore = !B.base_ignore || B.base_ignore[r];
      u.cpres = u.base_ignore ? 0u : (uniform_u32(B.base_pres[r]) & u.allmask);
#pragma unroll
      for (int d = 0; d < DMAX; ++d) {
        u.S[d] = (d < (int)nd && ((u.spres >> d) & 1u)) ? uniform_u64(B.read_vc[(uint64_t)d * rstride + ridx]) : 0;
        u.C0[d] = (d < (int)nd && ((u.cpres >> d) & 1u)) ? uniform_u64(B.base_vc[(uint64_t)d * n + r]) : 0;
      }
      u.has_txid = B.txid && (!B.txid_valid || B.txid_valid[r]) && L.op_txid;
      u.txid = u.has_txid ? uniform_u64(B.txid[r]) : 0;
      if (PACKED) pk_setup(u, nd, uniform_u64(L.key_tbase[uniform_u64(B.key[r])]), pk);
      ap.reset();
      a.reset();
    }
    const uint64_t t0 = R0.off0 & ~(uint64_t)(OPL - 1), c = x - R0.gchunk0;
    const uint64_t lo = t0 + c * CHUNK, hi = lo + CHUNK < R0.off1 ? lo + CHUNK : R0.off1;
    const uint64_t g = lo + (uint64_t)tid * OPL;
    if (TYPE == AM_BCOUNTER) {  // included ops -> LDS slot sums (orddict:update_counter)
      if (g < hi) {
        const uint32_t meta4 = *(const uint32_t *)(L.op_meta + g);
        const uint32_t ib = LEAN ? lean_incl4<DMAX>(L, nd, stride, u, pk, lr, vS, g, R0.off0, hi, ap, a, emx)
                                 : incl4<DMAX, PACKED>(L, nd, stride, u, pk, g, R0.off0, hi, ap, a);
#pragma unroll
        for (int k = 0; k < OPL; ++k) {
          if (!((ib >> k) & 1u)) continue;
          const uint32_t meta = (meta4 >> (8 * k)) & 0xFFu;
          if (meta & AM_META_BAD) continue;  // reported through FLAG_BAD
          uint32_t slot;
          int64_t v;
          if (!bc_slot(L, g + k, meta, nd, slot, v)) {
            a.flags |= FLAG_BAD;
            continue;
          }
          acc128_atomic(&slo[slot], &shi[slot], v < 0 ? -1 : 0, (uint64_t)v);
          atomicOr(&spres[slot], 1u);
        }
      }
      continue;  // the slot sums stay in LDS until the read's flush
    }
    for (uint32_t i = tid; i < 2 * GH; i += BLOCK) hs[i] = GH_EMPTY;
    if (tid < CHUNK / 32) incl[tid] = 0;
    __syncthreads();
    if (g < hi) {
      const uint32_t ib = LEAN ? lean_incl4<DMAX>(L, nd, stride, u, pk, lr, vS, g, R0.off0, hi, ap, a, emx)
                               : incl4<DMAX, PACKED>(L, nd, stride, u, pk, g, R0.off0, hi, ap, a);
      if (ib) atomicOr(&incl[(uint32_t)(g - lo) >> 5], ib << ((uint32_t)(g - lo) & 31u));
    }
    __syncthreads();
    grouped_records(L, B.key[R0.r], R0, lo, hi, incl, hs, bm + R0.bm0, tid);
    __syncthreads();
  }
  if (cur != 0xFFFFFFFFu) flush();
}

// ---- grouped MV reads in two passes (no barrier-bound per-chunk pipeline):
//      k_big_gincl  runs of chunks: the ops' inclusion bits into a global bitmap (32 words per
//                   1024-op chunk, every word written) + the scalar partials, one reduction per
//                   read and workgroup -- a streaming kernel with no LDS state
//      k_big_grec   per chunk: the records against those bits, the chunk's births and kills
//                   settled in the LDS hash sets (grouped_records), the rest exported ----
//      LEAN (packed view, the batch clock: no bases / TxIds / op presence): the clock is read
//      once, the chunk loop tests the packed entries only, and an escaped op is evaluated one DC
//      at a time with its LastOpCt maxima into LDS -- no D-wide u64 arrays in the loop (D = 16:
//      227 -> fewer VGPRs)
template <int DMAX, bool PACKED, bool LEAN = false>
__global__ void __launch_bounds__(BLOCK) k_big_gincl(am_op_log L, am_read_batch B, const uint32_t *nbig_p,
                                                     const BigRead *br, BigAcc *accs, uint32_t *ibm, uint64_t n_gch) {
  static_assert(!LEAN || PACKED, "the lean pass reads the packed view");
  __shared__ uint64_t red[BLOCK / WAVE][DMAX + 4];
  __shared__ unsigned long long emx[DMAX];  // LEAN: the read's escaped ops' LastOpCt maxima
  const uint32_t tid = threadIdx.x, lane = tid & (WAVE - 1), wv = tid / WAVE;
  const uint32_t nbig = uniform_u32(*nbig_p);
  const uint32_t nd = L.n_dc;
  const uint64_t stride = L.snap_stride ? L.snap_stride : L.n_ops;
  const uint64_t per = (n_gch + gridDim.x - 1) / gridDim.x;
  const uint64_t x0 = (uint64_t)blockIdx.x * per < n_gch ? (uint64_t)blockIdx.x * per : n_gch;
  const uint64_t x1 = x0 + per < n_gch ? x0 + per : n_gch;
  uint32_t cur = 0xFFFFFFFFu;
  BigRead R0{};
  ReadU<DMAX> u;
  PkRead<DMAX> pk;
  AccP<DMAX> ap;
  Acc<DMAX> a;
  uint64_t vS = 0;  // LEAN: lane d holds the clock's entry d
  LagRead<DMAX> lr;  // LEAN: the read's lag bases (the lag view, when the store has one)
  lr.on = false;
  auto flush = [&]() {
    uint64_t mx[DMAX];
    wave_partials<DMAX, PACKED, LEAN>(ap, pk, u, nd, a, mx);
    const uint32_t cnt = wave_sum_u32(a.count), fl = wave_or_u32(a.flags), pr = wave_or_u32(a.pres);
    const uint64_t mn = wave_min_u64(a.min_excl);
    if (lane == 0) {
      red[wv][0] = cnt, red[wv][1] = fl, red[wv][2] = pr, red[wv][3] = mn;
#pragma unroll
      for (int d = 0; d < DMAX; ++d) red[wv][4 + d] = mx[d];
    }
    __syncthreads();
    if (tid < 4 + (uint32_t)DMAX) {
      uint64_t v = red[0][tid];
      for (uint32_t w = 1; w < BLOCK / WAVE; ++w) {
        const uint64_t y = red[w][tid];
        v = tid == 0 ? v + y : (tid <= 2 ? (v | y) : tid == 3 ? (v < y ? v : y) : (v > y ? v : y));
      }
      if (LEAN && tid >= 4) v = v > emx[tid - 4] ? v : emx[tid - 4];
      BigAcc *acc = accs + cur;
      if (tid == 0 && v) atomicAdd(&acc->count, (uint32_t)v);
      if (tid == 1 && v) atomicOr(&acc->flags, (uint32_t)v);
      if (tid == 2 && v) atomicOr(&acc->pres, (uint32_t)v);
      if (tid == 3 && v != NONE) atomicMin(&acc->min_excl, (unsigned long long)v);
      if (tid >= 4 && tid - 4 < nd && v) atomicMax(&acc->mx[tid - 4], (unsigned long long)v);
    }
    __syncthreads();
  };
  if constexpr (LEAN) lean_clock<DMAX>(B, nd, lane, u, vS);
  for (uint64_t x = x0; x < x1; ++x) {
    const bool same = cur != 0xFFFFFFFFu && x < R0.gchunk0 + ((R0.off1 - (R0.off0 & ~(uint64_t)(OPL - 1)) + CHUNK - 1) / CHUNK);
    const uint32_t b = same ? cur : find_read(br, nbig, x, [](const BigRead &v) { return v.gchunk0; });
    if (b != cur && LEAN) {
      if (cur != 0xFFFFFFFFu) flush();
      cur = b;
      R0 = br[b];
      if (tid < DMAX) emx[tid] = 0;
      __syncthreads();
      const uint64_t key = uniform_u64(B.key[R0.r]);
      pk_setup(u, nd, uniform_u64(L.key_tbase[key]), pk);
      lag_setup(L, nd, key, L.lag_ct != nullptr, lr);
      ap.reset();
      a.reset();
    } else if (b != cur) {
      if (cur != 0xFFFFFFFFu) flush();
      cur = b;
      R0 = br[b];
      const uint64_t r = R0.r;
      const uint64_t n = B.n_reads;
      u.allmask = nd >= 32 ? 0xFFFFFFFFu : ((1u << nd) - 1u);
      const uint64_t rstride = B.per_read_clock ? n : 1, ridx = B.per_read_clock ? r : 0;
      u.spres = uniform_u32(B.read_pres[ridx]) & u.allmask;
      u.base_ignore = !B.base_ignore || B.base_ignore[r];
      u.cpres = u.base_ignore ? 0u : (uniform_u32(B.base_pres[r]) & u.allmask);
#pragma unroll
      for (int d = 0; d < DMAX; ++d) {
        u.S[d] = (d < (int)nd && ((u.spres >> d) & 1u)) ? uniform_u64(B.read_vc[(uint64_t)d * rstride + ridx]) : 0;
        u.C0[d] = (d < (int)nd && ((u.cpres >> d) & 1u)) ? uniform_u64(B.base_vc[(uint64_t)d * n + r]) : 0;
      }
      u.has_txid = B.txid && (!B.txid_valid || B.txid_valid[r]) && L.op_txid;
      u.txid = u.has_txid ? uniform_u64(B.txid[r]) : 0;
      if (PACKED) pk_setup(u, nd, uniform_u64(L.key_tbase[uniform_u64(B.key[r])]), pk);
      ap.reset();
      a.reset();
    }
    const uint64_t t0 = R0.off0 & ~(uint64_t)(OPL - 1), c = x - R0.gchunk0;
    const uint64_t lo = t0 + c * CHUNK, hi = lo + CHUNK < R0.off1 ? lo + CHUNK : R0.off1;
    const uint64_t g = lo + (uint64_t)tid * OPL;
    uint32_t ib = 0;
    if (g < hi)
      ib = LEAN ? lean_incl4<DMAX>(L, nd, stride, u, pk, lr, vS, g, R0.off0, hi, ap, a, emx)
                : incl4<DMAX, PACKED>(L, nd, stride, u, pk, g, R0.off0, hi, ap, a);
    uint32_t word = ib << (OPL * (tid % 8));  // 8 lanes of 4 ops per 32-bit word
    word |= (uint32_t)__shfl_xor((int)word, 1);
    word |= (uint32_t)__shfl_xor((int)word, 2);
    word |= (uint32_t)__shfl_xor((int)word, 4);
    if (tid % 8 == 0) ibm[x * (CHUNK / 32) + tid / 8] = word;
  }
  if (cur != 0xFFFFFFFFu) flush();
}

__global__ void __launch_bounds__(BLOCK) k_big_grec(am_op_log L, am_read_batch B, const uint32_t *nbig_p,
                                                    const BigRead *br, const uint32_t *ibm, uint32_t *bm,
                                                    uint64_t n_gch) {
  __shared__ uint32_t hs[2 * GH];
  const uint32_t tid = threadIdx.x;
  const uint32_t nbig = uniform_u32(*nbig_p);
  const uint64_t per = (n_gch + gridDim.x - 1) / gridDim.x;
  const uint64_t x0 = (uint64_t)blockIdx.x * per < n_gch ? (uint64_t)blockIdx.x * per : n_gch;
  const uint64_t x1 = x0 + per < n_gch ? x0 + per : n_gch;
  uint32_t cur = 0xFFFFFFFFu;
  BigRead R0{};
  for (uint64_t x = x0; x < x1; ++x) {
    const bool same = cur != 0xFFFFFFFFu && x < R0.gchunk0 + ((R0.off1 - (R0.off0 & ~(uint64_t)(OPL - 1)) + CHUNK - 1) / CHUNK);
    if (!same) {
      cur = find_read(br, nbig, x, [](const BigRead &v) { return v.gchunk0; });
      R0 = br[cur];
    }
    const uint64_t t0 = R0.off0 & ~(uint64_t)(OPL - 1), c = x - R0.gchunk0;
    const uint64_t lo = t0 + c * CHUNK, hi = lo + CHUNK < R0.off1 ? lo + CHUNK : R0.off1;
    for (uint32_t i = tid; i < 2 * GH; i += BLOCK) hs[i] = GH_EMPTY;
    __syncthreads();
    grouped_records(L, B.key[R0.r], R0, lo, hi, ibm + x * (CHUNK / 32), hs, bm + R0.bm0, tid);
    __syncthreads();
  }
}

// ---- births -> hash on the kill key ----
template <int TYPE>
__global__ void k_big_hash(const uint32_t *nbig_p, const BigRead *br, const BigAcc *accs, BigRec G, uint64_t total) {
  const uint32_t nbig = *nbig_p;
  for (uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; x < total;
       x += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t b = find_read(br, nbig, x, [](const BigRead &v) { return v.rec0; });
    const BigRead R0 = br[b];
    const uint64_t i = x - R0.rec0;
    if (i >= accs[b].nbirth) continue;
    uint64_t qa, qb;
    birth_kill_key<TYPE>(G.ba[x], G.bb[x], qa, qb);
    uint64_t h = key_hash(qa, qb) & R0.hmask;
    while (atomicCAS(&G.H[R0.h0 + h], HEMPTY, (uint32_t)i) != HEMPTY) h = (h + 1) & R0.hmask;
  }
}

// ---- kills probe the hash: same key and an earlier birth -> dead ----
template <int TYPE>
__global__ void k_big_kill(const uint32_t *nbig_p, const BigRead *br, const BigAcc *accs, BigRec G, uint64_t total) {
  const uint32_t nbig = *nbig_p;
  for (uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; x < total;
       x += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t b = find_read(br, nbig, x, [](const BigRead &v) { return v.rec0; });
    const BigRead R0 = br[b];
    if (x - R0.rec0 >= accs[b].nkill) continue;
    const uint64_t qa = G.ka[x], qb = G.kb[x];
    const int32_t kp = G.kp[x];
    uint64_t h = key_hash(qa, qb) & R0.hmask;
    while (true) {
      const uint32_t i = G.H[R0.h0 + h];
      if (i == HEMPTY) break;
      const uint64_t y = R0.rec0 + i;
      uint64_t ba, bb;
      birth_kill_key<TYPE>(G.ba[y], G.bb[y], ba, bb);
      if (ba == qa && bb == qb && G.bp[y] < kp) G.dead[y] = 1;
      h = (h + 1) & R0.hmask;
    }
  }
}

// ---- finish: survivors sorted + CSR, scalar outputs ----
struct FinSmem {
  uint64_t oa[SCAP], ob[SCAP], ot[SCAP];
  int32_t oi[SCAP];
  uint32_t ctr[8];
  uint64_t red[4];
};

template <int DMAX, int TYPE>
__global__ void __launch_bounds__(BLOCK) k_big_finish(am_op_log L, am_read_batch B, am_read_result R,
                                                      const uint32_t *nbig_p, const BigRead *br, const BigAcc *accs,
                                                      BigRec G, BigSlots SL) {
  __shared__ FinSmem s;
  const uint32_t tid = threadIdx.x;
  const uint32_t nbig = uniform_u32(*nbig_p);
  const uint64_t n = B.n_reads;
  const uint32_t nd = L.n_dc;
  for (uint32_t b = blockIdx.x; b < nbig; b += gridDim.x) {
    const BigRead R0 = br[b];
    const BigAcc A = accs[b];
    const uint64_t r = R0.r;
    int32_t status = (A.flags & FLAG_BAD) ? AM_ERR_UNEXPECTED_OPERATION : AM_OK;
    if (TYPE == AM_BCOUNTER && status == AM_OK) {
      const uint32_t np = nd * nd;
      uint32_t ovf = 0;
      for (uint32_t i = tid; i < SL.ns; i += BLOCK) {
        const uint64_t q = (uint64_t)b * SL.ns + i;
        if (SL.hi[q] != ((int64_t)SL.lo[q] < 0 ? -1 : 0)) ovf = 1;
      }
      ovf = (uint32_t)block_red_u64(s.red, wave_or_u32(ovf), 1);
      (void)np;
      if (ovf) {
        status = AM_ERR_OVERFLOW;  // Erlang: a bignum
      } else {
        if (tid < WAVE) {  // one wave compacts the present slots into the read's CSR range
          const uint64_t q0 = (uint64_t)b * SL.ns;
          const uint32_t ne = bc_emit<WAVE>(R, r, SL.ns, tid, 0, [&](uint32_t k, int64_t &v) {
            v = (int64_t)SL.lo[q0 + k];
            return SL.pres[q0 + k] != 0;
          });
          if (tid == 0) s.ctr[7] = ne;
        }
        __syncthreads();
        const uint32_t ne = s.ctr[7];
        if (ne > R.value.set_off[r + 1] - R.value.set_off[r]) status = AM_ERR_CAPACITY;
        else if (tid == 0) R.value.set_len[r] = ne;
        __syncthreads();
      }
    } else if (TYPE == AM_MVREG && status == AM_OK && R0.grouped) {
      // grouped mode: survivors = born & ~killed, already in output order (group order)
      const uint32_t gw = (R0.G + 31) / 32, lane = tid & 63u, wv = tid >> 6;
      const uint32_t *born = G.bm + R0.bm0, *killed = born + gw;
      const uint64_t ooff = R.value.set_off[r], ocap = R.value.set_off[r + 1] - ooff;
      const uint64_t rk0 = L.rec_key_off[B.key[r]];
      // FW consecutive words per thread: a hot key's bitmaps (tens of thousands of words) take
      // a few rounds of loads, not one round per 256 words
      constexpr uint32_t FW = 8;
      uint32_t base = 0;
      for (uint32_t w0 = 0; w0 < gw; w0 += BLOCK * FW) {
        const uint32_t wt = w0 + tid * FW;
        uint32_t a[FW], c = 0;
#pragma unroll
        for (uint32_t k = 0; k < FW; ++k) {
          a[k] = wt + k < gw ? (born[wt + k] & ~killed[wt + k]) : 0u;
          c += (uint32_t)__popc(a[k]);
        }
        const uint32_t inc = wave_incl_scan_u32(c, lane);
        if (lane == 63) s.ctr[wv] = inc;
        __syncthreads();
        uint32_t woff = 0, tot = 0;
        for (uint32_t v = 0; v < BLOCK / WAVE; ++v) {
          if (v < wv) woff += s.ctr[v];
          tot += s.ctr[v];
        }
        uint64_t o = base + woff + inc - c;
        for (uint32_t k = 0; k < FW; ++k)
          for (uint32_t bits = a[k]; bits && o < ocap; bits &= bits - 1, ++o) {
            const uint64_t g = (uint64_t)(wt + k) * 32 + (uint32_t)__builtin_ctz(bits);
            const u64x2 pr = *(const u64x2 *)(L.grp + 2 * (rk0 + g));
            R.value.set_a[ooff + o] = pr.x, R.value.set_b[ooff + o] = pr.y;
          }
        base += tot;
        __syncthreads();
      }
      if (base > ocap) status = AM_ERR_CAPACITY;
      else if (tid == 0) R.value.set_len[r] = base;
    } else if (status == AM_OK) {
      // count survivors, then gather them (LDS, or the read's kill records as scratch)
      uint32_t alive = 0;
      for (uint32_t i = tid; i < A.nbirth; i += BLOCK) alive += G.dead[R0.rec0 + i] ? 0u : 1u;
      alive = (uint32_t)block_red_u64(s.red, wave_sum_u32(alive), 0);
      const bool in_lds = alive <= SCAP;
      uint64_t *oa = in_lds ? s.oa : G.ka + R0.rec0;
      uint64_t *ob = in_lds ? s.ob : G.kb + R0.rec0;
      uint64_t *ot = in_lds ? s.ot : G.ot + R0.rec0;
      int32_t *oi = in_lds ? s.oi : G.oi + R0.rec0;
      if (tid == 0) s.ctr[0] = 0;
      __syncthreads();
      for (uint32_t i0 = 0; i0 < A.nbirth; i0 += BLOCK) {  // stable-order compaction is not
        const uint32_t i = i0 + tid;                         // needed: the sort follows
        if (i < A.nbirth && !G.dead[R0.rec0 + i]) {
          const uint32_t o = atomicAdd(&s.ctr[0], 1u);
          const uint64_t y = R0.rec0 + i;
          oa[o] = G.ba[y];
          if (TYPE == AM_AWSET) {  // (elem, newest birth first, token order); base last
            ob[o] = ((uint64_t)(uint32_t)(0x7FFFFFFF - G.bp[y]) << 32) | G.bs[y];
            ot[o] = G.bb[y];
            oi[o] = (int32_t)o;
          } else {
            ob[o] = G.bb[y];
          }
        }
      }
      __syncthreads();
      const uint64_t ooff = R.value.set_off[r], ocap = R.value.set_off[r + 1] - ooff;
      uint32_t distinct;
      if (TYPE == AM_AWSET) {
        block_sort(oa, ob, oi, alive, in_lds ? SCAP : (uint32_t)R0.cap);
        for (uint32_t j = tid; j < alive && j < ocap; j += BLOCK) {
          R.value.set_a[ooff + j] = oa[j];
          R.value.set_b[ooff + j] = ot[oi[j]];
        }
        distinct = alive;
      } else {
        block_sort(oa, ob, nullptr, alive, in_lds ? SCAP : (uint32_t)R0.cap);
        distinct = block_write_unique(oa, ob, alive, R.value.set_a + ooff, R.value.set_b + ooff, ocap, &s.ctr[4]);
      }
      if (distinct > ocap) status = AM_ERR_CAPACITY;
      else if (tid == 0) R.value.set_len[r] = distinct;
    }
    if (tid == 0) {
      R.status[r] = status;
      R.flags[r] = (uint8_t)(A.flags & 0xFFu);
      if (status == AM_OK) {
        const uint64_t key = B.key[r];
        const uint64_t idb = L.key_id_base ? L.key_id_base[key] : 1;
        const uint64_t nops = R0.off1 - R0.off0;
        int64_t nlo;
        if (A.min_excl != NONE)
          nlo = (L.op_id ? (int64_t)L.op_id[A.min_excl] : (int64_t)(idb + (A.min_excl - R0.off0))) - 1;
        else
          nlo = nops == 0 ? 0 : (L.op_id ? (int64_t)L.op_id[R0.off1 - 1] : (int64_t)(idb + nops - 1));
        R.new_last_op[r] = nlo;
        const uint32_t allmask = nd >= 32 ? 0xFFFFFFFFu : ((1u << nd) - 1u);
        const bool base_ignore = !B.base_ignore || B.base_ignore[r];
        const uint32_t cpres = base_ignore ? 0u : (B.base_pres[r] & allmask);
        const bool ign = base_ignore && A.count == 0;
        const uint32_t opres = ign ? 0u : (A.pres | cpres);
        R.last_ct_ignore[r] = ign ? 1 : 0;
        R.last_ct_pres[r] = opres;
        for (uint32_t d = 0; d < nd; ++d) {
          const uint64_t c0 = ((cpres >> d) & 1u) ? B.base_vc[(uint64_t)d * n + r] : 0;
          const uint64_t m = A.mx[d] > c0 ? A.mx[d] : c0;
          R.last_ct[(uint64_t)d * n + r] = ((opres >> d) & 1u) ? m : 0;
        }
        R.is_new_ss[r] = A.count > 0;
        R.count[r] = A.count;
      }
    }
    __syncthreads();
  }
}

template <int DMAX, int TYPE>
int run_big(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, const uint32_t *list,
            const uint32_t *nbig_d, uint32_t nbig, BigRead *br, BigAcc *acc, BigRec G, BigSlots SL,
            uint64_t n_chunks, uint64_t n_rec, uint64_t n_gch) {
  const uint32_t cap = (uint32_t)ctx->n_cu * 2;
  static bool attr = false;
  if (!attr) {
    AM_HIP(hipFuncSetAttribute((const void *)k_big_chunk<DMAX, TYPE, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)sizeof(ChunkSmem)));
    AM_HIP(hipFuncSetAttribute((const void *)k_big_chunk<DMAX, TYPE, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)sizeof(ChunkSmem)));
    attr = true;
  }
  const unsigned g1 = (unsigned)(n_chunks < cap ? n_chunks : cap);
  if (g1) {
    if (am_log_packed(L))  // the packed view: u32 commit vectors (4 * n_dc bytes per op, not 8 + 8 * n_dc)
      hipLaunchKernelGGL((k_big_chunk<DMAX, TYPE, true>), dim3(g1), dim3(BLOCK), sizeof(ChunkSmem), ctx->stream, *L,
                         *B, nbig_d, br, acc, G, SL, n_chunks);
    else
      hipLaunchKernelGGL((k_big_chunk<DMAX, TYPE, false>), dim3(g1), dim3(BLOCK), sizeof(ChunkSmem), ctx->stream, *L,
                         *B, nbig_d, br, acc, G, SL, n_chunks);
    AM_HIP(hipGetLastError());
  }
  if constexpr (TYPE == AM_MVREG) if (n_gch) {  // grouped MV reads: inclusion pass, record pass
    const uint64_t gcap = (uint64_t)ctx->n_cu * 8;
    const unsigned g4 = (unsigned)(n_gch < gcap ? n_gch : gcap);
    if (am_log_packed(L) && !am_batch_general(L, B))
      hipLaunchKernelGGL((k_big_gincl<DMAX, true, true>), dim3(g4), dim3(BLOCK), 0, ctx->stream, *L, *B, nbig_d, br,
                         acc, G.ibm, n_gch);
    else if (am_log_packed(L))
      hipLaunchKernelGGL((k_big_gincl<DMAX, true>), dim3(g4), dim3(BLOCK), 0, ctx->stream, *L, *B, nbig_d, br, acc,
                         G.ibm, n_gch);
    else
      hipLaunchKernelGGL((k_big_gincl<DMAX, false>), dim3(g4), dim3(BLOCK), 0, ctx->stream, *L, *B, nbig_d, br, acc,
                         G.ibm, n_gch);
    const uint64_t rcap = (uint64_t)ctx->n_cu * 16;
    hipLaunchKernelGGL(k_big_grec, dim3((unsigned)(n_gch < rcap ? n_gch : rcap)), dim3(BLOCK), 0, ctx->stream, *L, *B,
                       nbig_d, br, G.ibm, G.bm, n_gch);
    AM_HIP(hipGetLastError());
  }
  if constexpr (TYPE == AM_BCOUNTER) if (n_gch) {  // runs of chunks: bounded-counter reads
    const uint64_t gcap = (uint64_t)ctx->n_cu * 8;
    const unsigned g4 = (unsigned)(n_gch < gcap ? n_gch : gcap);
    if (am_log_packed(L) && !am_batch_general(L, B))
      hipLaunchKernelGGL((k_big_run<DMAX, TYPE, true, true>), dim3(g4), dim3(BLOCK), 0, ctx->stream, *L, *B, nbig_d, br,
                         acc, G.bm, SL, n_gch);
    else if (am_log_packed(L))
      hipLaunchKernelGGL((k_big_run<DMAX, TYPE, true>), dim3(g4), dim3(BLOCK), 0, ctx->stream, *L, *B, nbig_d, br, acc,
                         G.bm, SL, n_gch);
    else
      hipLaunchKernelGGL((k_big_run<DMAX, TYPE, false>), dim3(g4), dim3(BLOCK), 0, ctx->stream, *L, *B, nbig_d, br,
                         acc, G.bm, SL, n_gch);
    AM_HIP(hipGetLastError());
  }
  if (TYPE != AM_BCOUNTER) {
    const uint64_t eg = (n_rec + 255) / 256;
    const unsigned g2 = (unsigned)(eg < (uint64_t)ctx->n_cu * 16 ? eg : (uint64_t)ctx->n_cu * 16);
    hipLaunchKernelGGL((k_big_hash<TYPE>), dim3(g2), dim3(256), 0, ctx->stream, nbig_d, br, acc, G, n_rec);
    AM_HIP(hipGetLastError());
    hipLaunchKernelGGL((k_big_kill<TYPE>), dim3(g2), dim3(256), 0, ctx->stream, nbig_d, br, acc, G, n_rec);
    AM_HIP(hipGetLastError());
  }
  const unsigned g3 = (unsigned)(nbig < cap ? nbig : cap);
  hipLaunchKernelGGL((k_big_finish<DMAX, TYPE>), dim3(g3), dim3(BLOCK), 0, ctx->stream, *L, *B, *R, nbig_d, br, acc,
                     G, SL);
  AM_HIP(hipGetLastError());
  return AM_OK;
}

template <int TYPE>
int launch_big(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_retry retry) {
  uint64_t h[2];
  int rc = am_ctx_fetch(ctx, retry.count, 1, h);  // one synchronization: the tier is data-dependent
  if (rc) return rc;
  const uint32_t nbig = (uint32_t)(h[0] & 0xFFFFFFFFu);
  if (nbig == 0) return AM_OK;
  // metadata: BigRead[nbig], BigAcc[nbig], sizes[2][nbig], totals[2], bcounter slots
  BigSlots SL;
  SL.ns = TYPE == AM_BCOUNTER ? L->n_dc * L->n_dc + L->n_dc : 0;
  const size_t o_acc = am_round_up((size_t)nbig * sizeof(BigRead), 256);
  const size_t o_sz = o_acc + am_round_up((size_t)nbig * sizeof(BigAcc), 256);
  const size_t o_tot = o_sz + am_round_up((size_t)nbig * 32, 256);
  const size_t o_slo = o_tot + 256, nsl = (size_t)nbig * SL.ns;
  const size_t o_shi = o_slo + am_round_up(nsl * 8, 256), o_spr = o_shi + am_round_up(nsl * 8, 256);
  void *meta = nullptr;
  rc = am_ctx_scratch(ctx, AM_SCR_BIGMETA, o_spr + am_round_up(nsl * 4, 256) + 256, &meta);
  if (rc) return rc;
  BigRead *br = (BigRead *)meta;
  BigAcc *acc = (BigAcc *)((char *)meta + o_acc);
  uint64_t *sz = (uint64_t *)((char *)meta + o_sz);
  uint64_t *tot = (uint64_t *)((char *)meta + o_tot);
  SL.lo = (uint64_t *)((char *)meta + o_slo);
  SL.hi = (int64_t *)((char *)meta + o_shi);
  SL.pres = (uint32_t *)((char *)meta + o_spr);
  const uint64_t gq = ((uint64_t)nbig * SL.ns + 255) / 256, gcap = (uint64_t)ctx->n_cu * 8;
  const unsigned gp = (unsigned)std::max<uint64_t>((nbig + 255) / 256, gq < gcap ? gq : gcap);
  hipLaunchKernelGGL(k_big_prep<TYPE>, dim3(gp), dim3(256), 0, ctx->stream, *L, *B, retry.list, retry.count, br, acc,
                     sz, SL);
  AM_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_big_offsets, dim3(1), dim3(1024), 0, ctx->stream, retry.count, br, sz, tot);
  AM_HIP(hipGetLastError());
  uint64_t t4[4];
  rc = am_ctx_fetch(ctx, tot, 4, t4);
  if (rc) return rc;
  const uint64_t n_chunks = t4[0], n_rec = t4[1], n_bm = t4[2], n_gch = t4[3];
  // records: births (a, b, p, sub, dead), kills (a, b, p) -- n_rec each; hash 2*n_rec
  // slots; the finish pass's AW token / index scratch -- n_rec each
  const size_t rb = am_round_up(n_rec * 8, 256), r4 = am_round_up(n_rec * 4, 256), r1 = am_round_up(n_rec, 256);
  const size_t hb = am_round_up(2 * n_rec * 4, 256), bmb = am_round_up(n_bm * 4 + 4, 256);
  const size_t ib = TYPE == AM_MVREG ? am_round_up(n_gch * (CHUNK / 32) * 4 + 4, 256) : 0;
  void *recs = nullptr;
  rc = am_ctx_scratch(ctx, AM_SCR_BIGREC, 5 * rb + 4 * r4 + r1 + hb + bmb + ib, &recs);
  if (rc) return rc;
  char *q = (char *)recs;
  BigRec G;
  G.ba = (uint64_t *)q, q += rb;
  G.bb = (uint64_t *)q, q += rb;
  G.ka = (uint64_t *)q, q += rb;
  G.kb = (uint64_t *)q, q += rb;
  G.bp = (int32_t *)q, q += r4;
  G.kp = (int32_t *)q, q += r4;
  G.bs = (uint32_t *)q, q += r4;
  G.ot = (uint64_t *)q, q += rb;
  G.oi = (int32_t *)q, q += r4;
  G.dead = (uint8_t *)q, q += r1;
  G.H = (uint32_t *)q, q += hb;
  G.bm = (uint32_t *)q, q += bmb;
  G.ibm = (uint32_t *)q;
  if (n_bm) AM_HIP(hipMemsetAsync(G.bm, 0, n_bm * 4, ctx->stream));
  AM_HIP(hipMemsetAsync(G.dead, 0, n_rec, ctx->stream));
  AM_HIP(hipMemsetAsync(G.H, 0xFF, 2 * n_rec * 4, ctx->stream));
  const uint32_t nd = L->n_dc;
#define AM_B(D) \
  return run_big<D, TYPE>(ctx, L, B, R, retry.list, retry.count, nbig, br, acc, G, SL, n_chunks, n_rec, n_gch);
  if (nd <= 1) AM_B(1)
  if (nd <= 2) AM_B(2)
  if (nd <= 3) AM_B(3)
  if (nd <= 4) AM_B(4)
  if (nd <= 8) AM_B(8)
  if (nd <= 16) AM_B(16)
  AM_B(32)
#undef AM_B
}

}  // namespace

int am_launch_big(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, uint32_t type,
                  am_retry retry) {
  if (!retry.count) return AM_OK;
  switch (type) {
    case AM_AWSET: return launch_big<AM_AWSET>(ctx, L, B, R, retry);
    case AM_MVREG: return launch_big<AM_MVREG>(ctx, L, B, R, retry);
    case AM_BCOUNTER: return launch_big<AM_BCOUNTER>(ctx, L, B, R, retry);
    default: return AM_OK;
  }
}
