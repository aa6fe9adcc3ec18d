// am_snapcache.hip -- the materializer_vnode snapshot cache on the device, so a batch of
// reads runs the whole of materializer_vnode:internal_read/7 (src/materializer_vnode.erl:
// 371-376) without leaving HBM:
//   k_sc_claim     one read per key and batch (the lowest read index owns the key)
//   k_sc_select    get_from_snapshot_cache/5 (:384-413): no dict yet -> base {ignore,
//                  new()} and is_newest = true; otherwise vector_orddict:get_smaller/2
//                  (src/vector_orddict.erl:75-87): the newest cached snapshot whose
//                  clock is vectorclock:le the read clock; none -> the log cold path
//   am_materialize materialize/4 on the selected bases (every tier of am_plan.hip)
//   k_sc_store     the empty-dict insertion of get_from_snapshot_cache, then
//                  materialize_snapshot/7's write-back (:469-509): only when the key has
//                  ops, LastOpCt /= ignore, and (WasUpdated, IsNewest and Count >=
//                  MIN_OP_STORE_SS) or ShouldGC; internal_store_ss/4 (:342-364) with its
//                  NewLastOp - first.last_op_id >= MIN_OP_STORE_SS test (or ShouldGC);
//                  vector_orddict:insert_bigger/3 (:127-140); snapshot_insert_gc/4
//                  (:515-563): at SNAPSHOT_THRESHOLD entries, or on ShouldGC, the dict
//                  keeps its newest SNAPSHOT_MIN entries and the key's prune threshold
//                  (vectorclock:min over them) is emitted for prune_ops (am_store_update)
//   k_sc_release   frees the key claims
// Layout: per key a fixed array of CAP entries, newest first (clock [n_dc] + presence,
// last_op_id, value), entry-major: field[e][key] (clocks [e][d][key]), so a batch's reads of
// consecutive keys touch consecutive words of every field.  Scalar values (PN counter, LWW register) live in the entry; set
// values (add-wins set / MV register pairs) and bounded-counter (slot, value) entries live in
// a value pool (pool_a / pool_b words, bump-allocated, compacted on the host side when a batch
// could overflow it) that the next read's base points into (base.set_off/set_len), so a
// cached base is never copied.
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "am_wave.h"

using namespace amk;

struct am_snapcache {
  am_ctx *ctx = nullptr;
  uint32_t n_dc = 0;
  uint64_t n_keys = 0;
  uint8_t *cnt = nullptr;      // [n_keys] entries; ABSENT: no snapshot dict yet
  uint32_t *owner = nullptr;   // [n_keys] batch claim (~0: free)
  uint64_t *vc = nullptr;      // [CAP][n_dc][n_keys]
  uint32_t *pres = nullptr;    // [CAP][n_keys]
  int64_t *last_op = nullptr;  // [CAP][n_keys]
  int64_t *v0 = nullptr;       // [CAP][n_keys]
  uint64_t *v1 = nullptr;      // [CAP][n_keys]
  uint8_t *vflag = nullptr;    // [CAP][n_keys]
  uint64_t *poff = nullptr;    // [CAP][n_keys] value words in the pool
  uint32_t *plen = nullptr;    // [CAP][n_keys]
  uint64_t *pool_a = nullptr, *pool_b = nullptr;  // set pairs (a, b); bcounter slot values in a
  uint8_t *pool_p = nullptr;                      // bcounter slot presence
  uint32_t *pool_g = nullptr;                     // set pairs: token-group hint (am_ctx::grp_hint_in)
  uint64_t pool_cap = 0;                          // words
  uint64_t *ctr = nullptr;     // device [0] pool words used
  // the last batch's stored value words end, per wave of k_sc_store (the pool counter advances
  // to their maximum at the next batch's k_sc_sizes, not by the batch's whole result capacity)
  uint64_t *wend = nullptr;
  uint32_t wend_n = 0;         // entries pending (0: consumed)
  std::vector<void *> allocs;
};

namespace {

constexpr uint32_t CAP = AM_SNAPSHOT_THRESHOLD;   // insert_bigger + gc keep at most THRESHOLD - 1
constexpr uint32_t SMIN = AM_SNAPSHOT_MIN;
constexpr uint32_t MIN_OP_STORE_SS = AM_MIN_OP_STORE_SS;
constexpr uint8_t ABSENT = 0xFF;
// per-read selection codes (scratch)
enum : uint8_t { SEL_CACHED = 0, SEL_NEW_DICT = 1, SEL_COLD = 2, SEL_DUP = 3, SEL_BAD = 4 };

struct ScView {  // kernel-side copy of the cache pointers
  uint32_t n_dc;
  uint64_t n_keys;
  uint8_t *cnt;
  uint32_t *owner;
  uint64_t *vc;
  uint32_t *pres;
  int64_t *last_op, *v0;
  uint64_t *v1;
  uint8_t *vflag;
  uint64_t *poff;
  uint32_t *plen;
  uint64_t *pool_a, *pool_b;
  uint8_t *pool_p;
  uint32_t *pool_g;
  uint64_t pool_cap;
  uint64_t *ctr;
};
// selected bases (scratch, columns of the batch handed to am_materialize)
struct ScSel {
  uint8_t *code, *newest, *base_ignore, *vflag;
  uint64_t *base_vc, *v1, *set_off;
  uint32_t *base_pres, *set_len;
  int64_t *base_last_op, *v0;
  uint64_t *cp_dst;  // k_sc_store -> k_sc_copy: the stored snapshot's value words go to pool
  uint32_t *cp_len;  //   words [cp_dst, cp_dst + cp_len) from the read's result CSR (0: none)
};
// prune thresholds emitted by snapshot_insert_gc (optional)
struct ScGc {
  uint8_t *mask;     // [n_keys]
  uint64_t *thr_vc;  // [n_dc][n_keys]
  uint32_t *thr_pres;
};

// entry e of key k: its field index, its clock entry d (entry-major layout)
__device__ __forceinline__ uint64_t ent(const ScView &C, uint32_t e, uint64_t k) { return (uint64_t)e * C.n_keys + k; }
__device__ __forceinline__ uint64_t vci(const ScView &C, uint32_t e, uint64_t k, uint32_t d) {
  return ((uint64_t)e * C.n_dc + d) * C.n_keys + k;
}
__device__ __forceinline__ uint64_t clk(const ScView &C, uint32_t e, uint64_t k, uint32_t pres, uint32_t d) {
  return ((pres >> d) & 1u) ? C.vc[vci(C, e, k, d)] : 0;
}

// snapshot_insert_gc/4's prune threshold (src/materializer_vnode.erl:523-527) over key k's
// kept entries [0, keep) (newest first): Acc = the oldest kept clock, then for every entry
// newest -> oldest Acc = vectorclock:min([CT1, Acc]), i.e. each DC of CT1 lowered to
// min(CT1[dc], Acc[dc]) with a DC missing from Acc read as 0 (a DC only in Acc keeps its entry;
// oracle/ref_materializer.py vc_min2 gives the evidence for this rule).  Writes thr[d * stride]
// (0 for absent DCs) and returns the presence mask.
__device__ uint32_t gc_threshold(const ScView &C, uint64_t k, uint32_t keep, uint64_t *thr, uint64_t stride) {
  const uint32_t nd = C.n_dc;
  const uint32_t last = keep - 1;
  uint32_t pres = 0;
  for (uint32_t d = 0; d < nd; ++d) {
    bool have = (C.pres[ent(C, last, k)] >> d) & 1u;
    uint64_t acc = have ? C.vc[vci(C, last, k, d)] : 0;
    for (uint32_t e = 0; e < keep; ++e) {
      if (!((C.pres[ent(C, e, k)] >> d) & 1u)) continue;
      const uint64_t a = C.vc[vci(C, e, k, d)], b = have ? acc : 0;
      acc = a < b ? a : b;
      have = true;
    }
    thr[(uint64_t)d * stride] = have ? acc : 0;
    pres |= (have ? 1u : 0u) << d;
  }
  return pres;
}

__global__ void k_sc_claim(ScView C, am_read_batch B) {
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < B.n_reads; r += (uint64_t)gridDim.x * blockDim.x)
    if (B.key[r] < C.n_keys) atomicMin(&C.owner[B.key[r]], (uint32_t)r);
}

__global__ void k_sc_release(ScView C, am_read_batch B) {
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < B.n_reads; r += (uint64_t)gridDim.x * blockDim.x)
    if (B.key[r] < C.n_keys) C.owner[B.key[r]] = 0xFFFFFFFFu;
}

__global__ void k_sc_select(ScView C, am_read_batch B, ScSel S) {
  const uint32_t nd = C.n_dc;
  const uint32_t all = nd >= 32 ? 0xFFFFFFFFu : ((1u << nd) - 1u);
  const uint64_t n = B.n_reads;
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t key = B.key[r];
    const uint32_t t = B.type[r];
    uint8_t code = SEL_NEW_DICT, newest = 1;
    uint32_t bpres = 0, blen = 0;
    int64_t blast = 0, bv0 = 0;
    uint64_t bv1 = 0, boff = 0;  // pool offset 0: the reserved zero words (new() bounded counter)
    uint8_t bvf = t == AM_LWW ? 1 : 0, bign = 1;  // new(): 0 / {0, <<>>} / [] / {[], []}
    uint32_t sel = CAP;
    if (key >= C.n_keys || t < AM_PN || t > AM_BCOUNTER) {
      code = SEL_BAD;
    } else if (C.owner[key] != (uint32_t)r) {
      code = SEL_DUP;
    } else if (C.cnt[key] != ABSENT) {
      const uint64_t ridx = B.per_read_clock ? r : 0, rstride = B.per_read_clock ? n : 1;
      const uint32_t spres = B.read_pres[ridx] & all;
      const uint32_t ne = C.cnt[key];
      for (uint32_t e = 0; e < ne && sel == CAP; ++e) {  // vector_orddict:get_smaller: newest first
        const uint32_t ep = C.pres[ent(C, e, key)] & all;
        bool le = true;  // vectorclock:le(Entry, ReadClock): every DC of either, missing = 0
        for (uint32_t d = 0; d < nd && le; ++d) {
          const uint64_t x = clk(C, e, key, ep, d);
          const uint64_t y = ((spres >> d) & 1u) ? B.read_vc[(uint64_t)d * rstride + ridx] : 0;
          le = x <= y;
        }
        if (le) sel = e;
      }
      if (sel == CAP) {
        code = SEL_COLD;  // get_from_snapshot_log: the log path, not the cache
      } else {
        const uint64_t slot = ent(C, sel, key);
        code = SEL_CACHED;
        newest = sel == 0;
        bign = 0;
        bpres = C.pres[slot] & all;
        for (uint32_t d = 0; d < nd; ++d) S.base_vc[(uint64_t)d * n + r] = clk(C, sel, key, bpres, d);
        blast = C.last_op[slot];
        bv0 = C.v0[slot];
        bv1 = C.v1[slot];
        bvf = C.vflag[slot];
        boff = C.poff[slot];
        blen = C.plen[slot];
      }
    }
    if (bign)
      for (uint32_t d = 0; d < nd; ++d) S.base_vc[(uint64_t)d * n + r] = 0;
    S.code[r] = code;
    S.newest[r] = newest;
    S.base_ignore[r] = bign;
    S.base_pres[r] = bpres;
    S.base_last_op[r] = blast;
    S.v0[r] = bv0;
    S.v1[r] = bv1;
    S.vflag[r] = bvf;
    S.set_off[r] = boff;
    S.set_len[r] = blen;  // set pairs; bounded counter (slot, value) entries
  }
}

// value words of read r's result (set pairs; bounded counter (slot, value) entries), or 0
// when the result columns are absent (not cached then)
__device__ __forceinline__ uint32_t value_words(const am_read_result &R, uint64_t r, uint32_t t, uint32_t nd) {
  (void)nd;
  if (t == AM_AWSET || t == AM_MVREG || t == AM_BCOUNTER)
    return (R.value.set_len && R.value.set_a && R.value.set_b) ? R.value.set_len[r] : 0u;
  return 0;
}

// Pool room: the batch reserved one pool word per result word (pool_reserve), so read r's
// snapshot goes to words [used + set_off[r] - set_off[0], + w) -- no atomics (one per read on
// one counter cost most of this kernel).  The group wave kernel already wrote the words there
// (tee_done[r]); k_sc_copy moves the others' from the result CSR.
__global__ void __launch_bounds__(256) k_sc_store(ScView C, am_op_log L, am_read_batch B, am_read_result R, ScSel S,
                                                  const uint8_t *should_gc, ScGc G, uint64_t used, uint64_t so0,
                                                  uint64_t *wend, const uint8_t *teed) {
  const uint32_t nd = C.n_dc;
  uint64_t wmax = 0;  // the end of the value words this wave stored (wend, or null: none reserved)
  const uint64_t n = B.n_reads;
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t rb = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); rb < n; rb += step) {
    const uint64_t r = rb + lane;
    bool act = r < n;  // this lane's read goes on to the write-back
    const uint8_t code = act ? S.code[r] : (uint8_t)SEL_BAD;
    if (act && code == SEL_BAD) {
      if (R.status[r] == AM_OK) R.status[r] = AM_ERR_INVALID;
      act = false;
    } else if (act && code == SEL_DUP) {
      R.status[r] = AM_ERR_INVALID;
      act = false;
    } else if (act && code == SEL_COLD) {
      R.status[r] = AM_ERR_COLD_PATH;  // get_from_snapshot_log: the log path, not the cache
      act = false;
    }
    const uint64_t key = act ? B.key[r] : 0;
    const uint32_t t = act ? B.type[r] : 0u;
    const uint64_t s0 = key;  // entry 0 of the key (entry e: ent(C, e, key))
    uint32_t ne = act ? C.cnt[key] : 0u;
    if (act && code == SEL_NEW_DICT) {  // store_snapshot(TxId, Key, Empty, vectorclock:new(), false)
      C.pres[s0] = 0;
      for (uint32_t d = 0; d < nd; ++d) C.vc[vci(C, 0, key, d)] = 0;
      C.last_op[s0] = 0;
      C.v0[s0] = 0;
      C.v1[s0] = 0;
      C.vflag[s0] = t == AM_LWW ? 1 : 0;
      C.poff[s0] = 0;
      C.plen[s0] = 0;
      ne = 1;
      C.cnt[key] = 1;
    }
    // materialize_snapshot/7: number_of_ops == 0 returns the base; errors and
    // CommitTime == ignore return without caching
    act = act && R.status[r] == AM_OK && am_kend(L, key) != L.key_off[key] && !R.last_ct_ignore[r];
    const bool sg = act && should_gc && should_gc[r];
    act = act && ((R.is_new_ss[r] && S.newest[r] && R.count[r] >= MIN_OP_STORE_SS) || sg);
    // internal_store_ss/4: ShouldInsert = NewLastOp - first.last_op_id >= MIN_OP_STORE_SS
    const int64_t nlo = act ? R.new_last_op[r] : 0;
    act = act && (nlo - C.last_op[s0] >= (int64_t)MIN_OP_STORE_SS || sg);
    // vector_orddict:insert_bigger: prepend iff not vectorclock:le(New, First)
    const uint32_t np = act ? R.last_ct_pres[r] : 0u;
    bool ins = false;
    if (act) {
      const uint32_t fp = C.pres[s0];
      bool le = true;
      for (uint32_t d = 0; d < nd && le; ++d) {
        const uint64_t x = ((np >> d) & 1u) ? R.last_ct[(uint64_t)d * n + r] : 0;
        le = x <= clk(C, 0, key, fp, d);
      }
      ins = !le;
    }
    // the value words' room in the pool (sized on the host before the batch; offset 0 is never
    // handed out): if it is ever missing the snapshot is not cached at all -- the read's own
    // result stands -- rather than cached with an empty value (ctr[1] records the event)
    const uint32_t w = ins ? value_words(R, r, t, nd) : 0u;
    uint64_t off = 0;
    if (w) {
      off = used + (R.value.set_off[r] - so0);
      if (off == 0 || off + w > C.pool_cap) {
        atomicOr((unsigned long long *)(C.ctr + 1), 1ull);
        ins = false;
        off = 0;
      }
    }
    if (act) {
      // snapshot_insert_gc/4: at SNAPSHOT_THRESHOLD entries (or ShouldGC) keep the newest
      // SNAPSHOT_MIN and prune the ops below their vectorclock:min
      const uint32_t grown = ne + (ins ? 1u : 0u);
      const bool gc = grown >= CAP || sg;
      const uint32_t keep = gc ? (grown < SMIN ? grown : SMIN) : grown;
      if (ins) {
        for (uint32_t e = keep - 1; e >= 1; --e) {  // shift right by one (newest first)
          const uint64_t dst = ent(C, e, key), src = ent(C, e - 1, key);
          for (uint32_t d = 0; d < nd; ++d) C.vc[vci(C, e, key, d)] = C.vc[vci(C, e - 1, key, d)];
          C.pres[dst] = C.pres[src];
          C.last_op[dst] = C.last_op[src];
          C.v0[dst] = C.v0[src];
          C.v1[dst] = C.v1[src];
          C.vflag[dst] = C.vflag[src];
          C.poff[dst] = C.poff[src];
          C.plen[dst] = C.plen[src];
        }
        for (uint32_t d = 0; d < nd; ++d) C.vc[vci(C, 0, key, d)] = ((np >> d) & 1u) ? R.last_ct[(uint64_t)d * n + r] : 0;
        C.pres[s0] = np;
        C.last_op[s0] = nlo;
        C.v0[s0] = (t == AM_PN || t == AM_LWW) ? R.value.v0[r] : 0;
        C.v1[s0] = t == AM_LWW ? R.value.v1[r] : 0;
        C.vflag[s0] = t == AM_LWW ? R.value.vflag[r] : 0;
        C.poff[s0] = off;
        C.plen[s0] = off ? w : 0;
      }
      C.cnt[key] = (uint8_t)keep;
      if (gc && G.mask) {  // the prune threshold over the kept entries
        G.thr_pres[key] = gc_threshold(C, key, keep, G.thr_vc + key, C.n_keys);
        G.mask[key] = 1;
      }
    }
    if (r < n) S.cp_dst[r] = off, S.cp_len[r] = (off && !(teed && teed[r])) ? w : 0u;
    if (ins && off) wmax = off + w > wmax ? off + w : wmax;
  }
  if (wend) {
    wmax = amk::wave_max_u64(wmax);
    if ((threadIdx.x & 63u) == 0) wend[(uint64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = wmax;
  }
}

// the value words (set pairs, bounded-counter entries) of stored snapshots the group wave
// kernel did not tee from the read's result CSR into the pool: 16 lanes per read, four reads
// per wave, coalesced (a thread copying a read's pairs serially cost C3's read/6 3.4 ms of 16;
// copying them inside k_sc_store, a read at a time per wave, 1.45 ms)
__global__ void k_sc_copy(ScView C, am_read_result R, ScSel S, uint64_t n) {
  const uint32_t sl = threadIdx.x & 15u;
  const uint64_t rows = (uint64_t)gridDim.x * (blockDim.x / 16);
  for (uint64_t r = (uint64_t)blockIdx.x * (blockDim.x / 16) + threadIdx.x / 16; r < n; r += rows) {
    const uint32_t w = S.cp_len[r];
    if (!w) continue;
    const uint64_t src = R.value.set_off[r], dst = S.cp_dst[r];
    for (uint32_t i = sl; i < w; i += 16) {
      C.pool_a[dst + i] = R.value.set_a[src + i], C.pool_b[dst + i] = R.value.set_b[src + i];
      C.pool_g[dst + i] = ~0u;  // no group hint
    }
  }
}

ScView view(const am_snapcache *c) {
  return ScView{c->n_dc, c->n_keys, c->cnt, c->owner, c->vc, c->pres, c->last_op, c->v0, c->v1, c->vflag,
                c->poff, c->plen, c->pool_a, c->pool_b, c->pool_p, c->pool_g, c->pool_cap, c->ctr};
}
unsigned grid(uint64_t n) { return (unsigned)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096); }

// forced snapshot_insert_gc/4 on every cached key (src/materializer_vnode.erl:519-536): the
// dict keeps its newest SNAPSHOT_MIN entries and the prune threshold is gc_threshold over them
__global__ void k_sc_threshold(ScView C, uint8_t *mask, uint64_t *thr_vc, uint32_t *thr_pres) {
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < C.n_keys;
       k += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t cnt = C.cnt[k];
    const uint32_t m = (cnt == ABSENT) ? 0 : (cnt < SMIN ? cnt : SMIN);
    if (cnt != ABSENT) C.cnt[k] = (uint8_t)m;
    thr_pres[k] = m ? gc_threshold(C, k, m, thr_vc + k, C.n_keys) : 0u;
    if (!m)
      for (uint32_t d = 0; d < C.n_dc; ++d) thr_vc[(uint64_t)d * C.n_keys + k] = 0;
    mask[k] = m ? 1 : 0;
  }
}

// ---- value pool compaction: the live entries' words moved to a fresh pool ----
__global__ void k_pool_len(ScView C, uint64_t *len) {
  const uint64_t ne = C.n_keys * CAP;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ne; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t k = i % C.n_keys, e = i / C.n_keys;
    const uint32_t cnt = C.cnt[k];
    len[i] = (cnt != ABSENT && e < cnt && C.poff[i]) ? C.plen[i] : 0;
  }
}
__global__ void k_pool_move(ScView C, const uint64_t *off, uint64_t base, uint64_t *na, uint64_t *nb, uint8_t *np,
                            uint32_t *ng) {
  const uint64_t ne = C.n_keys * CAP;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ne; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t k = i % C.n_keys, e = i / C.n_keys;
    const uint32_t cnt = C.cnt[k];
    if (cnt == ABSENT || e >= cnt || !C.poff[i]) continue;
    const uint64_t src = C.poff[i], dst = base + off[i];
    for (uint32_t j = 0; j < C.plen[i]; ++j)
      na[dst + j] = C.pool_a[src + j], nb[dst + j] = C.pool_b[src + j], np[dst + j] = C.pool_p[src + j],
               ng[dst + j] = C.pool_g[src + j];
    C.poff[i] = dst;
  }
}

// words at the pool start kept zero: a new() bounded counter's base (every slot absent)
uint64_t reserved_words(uint32_t nd) { return (uint64_t)nd * nd + nd + 1; }

// a batch's sizes in one readback: the result CSR's first and last offsets and the pool
// counters (words used, room-missing flag)
// The pool counter first advances past the previous batch's stored words (the max of its
// per-wave ends, nw of them).  One wave.
__global__ void k_sc_sizes(const uint64_t *set_off, uint64_t n, uint64_t *ctr, const uint64_t *wend, uint32_t nw,
                           uint64_t *out) {
  uint64_t m = 0;
  for (uint32_t i = threadIdx.x; i < nw; i += 64) m = wend[i] > m ? wend[i] : m;
  m = amk::wave_max_u64(m);
  if (threadIdx.x == 0) {
    const uint64_t used = m > ctr[0] ? m : ctr[0];
    ctr[0] = used;
    out[0] = set_off ? set_off[0] : 0;
    out[1] = set_off ? set_off[n] : 0;
    out[2] = used;
    out[3] = ctr[1];
  }
}

// at least `need` free pool words after the used ones (w = the pool counters as read by
// k_sc_sizes): compact, and grow when compaction does not free enough (synchronizes the stream)
int pool_reserve(am_snapcache *c, uint64_t need, const uint64_t w[2], uint64_t *used_out) {
  am_ctx *ctx = c->ctx;
  if (w[1]) {  // an earlier batch found its room missing (k_sc_store did not cache that snapshot)
    am_set_error("am_snapcache: a snapshot was not cached for lack of value-pool room (pool sizing)");
    return AM_ERR_NOMEM;
  }
  const uint64_t used = w[0];
  *used_out = used;
  if (used + need <= c->pool_cap) return AM_OK;
  const uint64_t ne = c->n_keys * CAP;
  uint64_t *len = nullptr;
  void *tmp = nullptr;
  size_t tmp_b = 0;
  if (hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_b, len, len, ne + 1, ctx->stream) != hipSuccess) return AM_ERR_HIP;
  AM_HIP(hipMalloc((void **)&len, (ne + 1) * 8));
  if (hipMalloc(&tmp, tmp_b + 16) != hipSuccess) {
    (void)hipFree(len);
    return AM_ERR_NOMEM;
  }
  ScView V = view(c);
  uint64_t live = 0;
  bool ok = hipMemsetAsync(len + ne, 0, 8, ctx->stream) == hipSuccess;
  if (ok && ne) {
    hipLaunchKernelGGL(k_pool_len, dim3(grid(ne)), dim3(256), 0, ctx->stream, V, len);
    ok = hipGetLastError() == hipSuccess;
  }
  ok = ok && hipcub::DeviceScan::ExclusiveSum(tmp, tmp_b, len, len, ne + 1, ctx->stream) == hipSuccess;
  if (ok) ok = am_ctx_fetch(ctx, len + ne, 1, &live) == AM_OK;
  const uint64_t res = reserved_words(c->n_dc);
  uint64_t cap = c->pool_cap;
  if (cap < 2 * (res + live + need)) cap = 2 * (res + live + need);  // grow: room for this batch twice
  uint64_t *na = nullptr, *nb = nullptr;
  uint8_t *np = nullptr;
  uint32_t *ng = nullptr;
  ok = ok && hipMalloc((void **)&na, cap * 8) == hipSuccess && hipMalloc((void **)&nb, cap * 8) == hipSuccess &&
       hipMalloc((void **)&np, cap) == hipSuccess && hipMalloc((void **)&ng, cap * 4) == hipSuccess;
  ok = ok && hipMemsetAsync(na, 0, res * 8, ctx->stream) == hipSuccess &&
       hipMemsetAsync(nb, 0, res * 8, ctx->stream) == hipSuccess && hipMemsetAsync(np, 0, res, ctx->stream) == hipSuccess &&
       hipMemsetAsync(ng, 0xFF, res * 4, ctx->stream) == hipSuccess;
  if (ok && ne) {
    hipLaunchKernelGGL(k_pool_move, dim3(grid(ne)), dim3(256), 0, ctx->stream, V, len, res, na, nb, np, ng);
    ok = hipGetLastError() == hipSuccess;
  }
  const uint64_t nused = res + live;
  *used_out = nused;
  ok = ok && hipMemcpyAsync(c->ctr, &nused, 8, hipMemcpyHostToDevice, ctx->stream) == hipSuccess &&
       hipStreamSynchronize(ctx->stream) == hipSuccess;
  (void)hipFree(len);
  (void)hipFree(tmp);
  if (!ok) {
    if (na) (void)hipFree(na);
    if (nb) (void)hipFree(nb);
    if (np) (void)hipFree(np);
    if (ng) (void)hipFree(ng);
    am_set_error("snapshot cache: value pool compaction failed");
    return AM_ERR_HIP;
  }
  (void)hipFree(c->pool_a);
  (void)hipFree(c->pool_b);
  (void)hipFree(c->pool_p);
  (void)hipFree(c->pool_g);
  c->pool_a = na, c->pool_b = nb, c->pool_p = np, c->pool_g = ng, c->pool_cap = cap;
  return AM_OK;
}


// relabelling (am_codec): LWW entry values in place; the pool words of set entries are
// marked first, so a pool word two entries share is relabelled once
__device__ __forceinline__ void sc_relabel_word(uint64_t *w, const uint64_t *old, const uint64_t *nw, uint64_t n) {
  const uint64_t x = *w;
  if (x == 0 || x == ~0ull) return;
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) / 2;
    if (old[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  if (lo < n && old[lo] == x) *w = nw[lo];
}

__global__ void k_sc_relabel_entries(const uint8_t *cnt, uint64_t n_keys, const uint8_t *ktype, const uint8_t *vflag,
                                     uint64_t *v1, const uint64_t *poff, const uint32_t *plen, uint32_t *mark,
                                     const uint64_t *old, const uint64_t *nw, uint64_t n) {
  for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n_keys * CAP; s += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t k = s % n_keys;  // entry-major: entry s / n_keys of key k
    if (cnt[k] == ABSENT || s / n_keys >= cnt[k]) continue;
    const uint32_t t = ktype[k];
    if (t == AM_LWW && !vflag[s]) sc_relabel_word(v1 + s, old, nw, n);
    if (t == AM_AWSET || t == AM_MVREG)
      for (uint64_t w = poff[s]; w < poff[s] + plen[s]; ++w) atomicOr(&mark[w / 32], 1u << (w % 32));
  }
}

__global__ void k_sc_relabel_pool(uint64_t *pa, uint64_t *pb, const uint32_t *mark, uint64_t words, const uint64_t *old,
                                  const uint64_t *nw, uint64_t n) {
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < words; w += (uint64_t)gridDim.x * blockDim.x)
    if ((mark[w / 32] >> (w % 32)) & 1u) {
      sc_relabel_word(pa + w, old, nw, n);
      sc_relabel_word(pb + w, old, nw, n);
    }
}

}  // namespace

extern "C" {

int am_snapcache_create(am_ctx *ctx, uint32_t n_dc, uint64_t n_keys, am_snapcache **out) {
  if (!ctx || !out || n_dc == 0 || n_dc > AM_MAX_DC) return AM_ERR_INVALID;
  AM_LOCK(ctx);
  AM_HIP(hipSetDevice(ctx->device));
  am_snapcache *c = new am_snapcache();
  c->ctx = ctx;
  c->n_dc = n_dc;
  c->n_keys = n_keys;
  const uint64_t ne = n_keys * CAP + 1;
  auto alloc = [&](size_t bytes, void **p) {
    int rc = am_dev_alloc(ctx, bytes, p);
    if (!rc) c->allocs.push_back(*p);
    return rc;
  };
  int rc = alloc(n_keys + 16, (void **)&c->cnt);
  if (!rc) rc = alloc((n_keys + 1) * 4, (void **)&c->owner);
  if (!rc) rc = alloc(ne * n_dc * 8, (void **)&c->vc);
  if (!rc) rc = alloc(ne * 4, (void **)&c->pres);
  if (!rc) rc = alloc(ne * 8, (void **)&c->last_op);
  if (!rc) rc = alloc(ne * 8, (void **)&c->v0);
  if (!rc) rc = alloc(ne * 8, (void **)&c->v1);
  if (!rc) rc = alloc(ne, (void **)&c->vflag);
  if (!rc) rc = alloc(ne * 8, (void **)&c->poff);
  if (!rc) rc = alloc(ne * 4, (void **)&c->plen);
  if (!rc) rc = alloc(16, (void **)&c->ctr);
  if (!rc) rc = alloc(4096 * 4 * 8, (void **)&c->wend);  // k_sc_store's grid (grid(): <= 4096 blocks of 4 waves)
  const uint64_t res = reserved_words(n_dc);
  c->pool_cap = 4 * res + 4096;
  if (!rc && (hipMalloc((void **)&c->pool_a, c->pool_cap * 8) != hipSuccess ||
              hipMalloc((void **)&c->pool_b, c->pool_cap * 8) != hipSuccess ||
              hipMalloc((void **)&c->pool_p, c->pool_cap) != hipSuccess ||
              hipMalloc((void **)&c->pool_g, c->pool_cap * 4) != hipSuccess))
    rc = AM_ERR_NOMEM;
  if (!rc && (hipMemsetAsync(c->cnt, ABSENT, n_keys + 16, ctx->stream) != hipSuccess ||
              hipMemsetAsync(c->owner, 0xFF, (n_keys + 1) * 4, ctx->stream) != hipSuccess ||
              hipMemsetAsync(c->poff, 0, ne * 8, ctx->stream) != hipSuccess ||
              hipMemsetAsync(c->plen, 0, ne * 4, ctx->stream) != hipSuccess ||
              hipMemsetAsync(c->pool_a, 0, res * 8, ctx->stream) != hipSuccess ||
              hipMemsetAsync(c->pool_b, 0, res * 8, ctx->stream) != hipSuccess ||
              hipMemsetAsync(c->pool_p, 0, res, ctx->stream) != hipSuccess ||
              hipMemsetAsync(c->pool_g, 0xFF, res * 4, ctx->stream) != hipSuccess ||
              hipMemcpyAsync(c->ctr, &res, 8, hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
              hipMemsetAsync(c->ctr + 1, 0, 8, ctx->stream) != hipSuccess ||
              hipStreamSynchronize(ctx->stream) != hipSuccess))
    rc = AM_ERR_HIP;
  if (rc) {
    am_snapcache_destroy(c);
    return rc;
  }
  *out = c;
  return AM_OK;
}

// a larger key space for the cache (keys [n_keys, new_n) start without a snapshot dict); the
// pool and every existing entry are kept
int am_snapcache_grow(am_snapcache *c, uint64_t new_n) {
  am_ctx *ctx = c->ctx;
  AM_LOCK(ctx);
  if (new_n <= c->n_keys) return AM_OK;
  const uint64_t nd = c->n_dc, n0 = c->n_keys, ne = new_n * CAP + 1;
  std::vector<void *> fresh;
  int rc = AM_OK;
  // rows = 1: a per-key column; rows = CAP (or CAP * n_dc): an entry-major field, whose rows of
  // n0 keys move to rows of new_n
  auto grow = [&](void **field, size_t w, size_t rows, size_t new_b, int fill) {
    void *p = nullptr;
    if (rc || (rc = am_dev_alloc(ctx, new_b, &p))) return;
    fresh.push_back(p);
    if (hipMemsetAsync(p, fill, new_b, ctx->stream) != hipSuccess ||
        (n0 && hipMemcpy2DAsync(p, new_n * w, *field, n0 * w, n0 * w, rows, hipMemcpyDeviceToDevice, ctx->stream) !=
                   hipSuccess))
      rc = AM_ERR_HIP;
    *field = p;
  };
  void *old[10] = {c->cnt, c->owner, c->vc, c->pres, c->last_op, c->v0, c->v1, c->vflag, c->poff, c->plen};
  grow((void **)&c->cnt, 1, 1, new_n + 16, ABSENT);
  grow((void **)&c->owner, 4, 1, (new_n + 1) * 4, 0xFF);
  grow((void **)&c->vc, 8, CAP * nd, ne * nd * 8, 0);
  grow((void **)&c->pres, 4, CAP, ne * 4, 0);
  grow((void **)&c->last_op, 8, CAP, ne * 8, 0);
  grow((void **)&c->v0, 8, CAP, ne * 8, 0);
  grow((void **)&c->v1, 8, CAP, ne * 8, 0);
  grow((void **)&c->vflag, 1, CAP, ne, 0);
  grow((void **)&c->poff, 8, CAP, ne * 8, 0);
  grow((void **)&c->plen, 4, CAP, ne * 4, 0);
  if (!rc && hipStreamSynchronize(ctx->stream) != hipSuccess) rc = AM_ERR_HIP;
  if (rc) {
    for (void *p : fresh) c->allocs.push_back(p);  // freed with the cache
    am_set_error("am_snapcache_grow failed");
    return rc;
  }
  for (void *p : old) {
    auto it = std::find(c->allocs.begin(), c->allocs.end(), p);
    if (it != c->allocs.end()) c->allocs.erase(it);
    am_dev_release(ctx, p);
  }
  for (void *p : fresh) c->allocs.push_back(p);
  c->n_keys = new_n;
  return AM_OK;
}

int am_snapcache_relabel(am_ctx *ctx, am_snapcache *c, const uint8_t *key_type, const uint64_t *old_labels,
                         const uint64_t *new_labels, uint64_t n) {
  if (!ctx || !c || c->ctx != ctx || !key_type || (n && (!old_labels || !new_labels))) return AM_ERR_INVALID;
  AM_LOCK(ctx);
  if (n == 0 || c->n_keys == 0) return AM_OK;
  AM_HIP(hipSetDevice(ctx->device));
  uint64_t *d_old = nullptr, *d_new = nullptr;
  if (int rc = am_relabel_upload(ctx, old_labels, new_labels, n, &d_old, &d_new)) return rc;
  uint32_t *mark = nullptr;
  const uint64_t mwords = c->pool_cap / 32 + 1;
  bool ok = hipMalloc((void **)&mark, mwords * 4) == hipSuccess &&
            hipMemsetAsync(mark, 0, mwords * 4, ctx->stream) == hipSuccess;
  if (ok) {
    const uint64_t ns = c->n_keys * CAP;
    hipLaunchKernelGGL(k_sc_relabel_entries, dim3((unsigned)std::min<uint64_t>((ns + 255) / 256, 65536)), dim3(256), 0,
                       ctx->stream, c->cnt, c->n_keys, key_type, c->vflag, c->v1, c->poff, c->plen, mark, d_old, d_new,
                       n);
    hipLaunchKernelGGL(k_sc_relabel_pool, dim3((unsigned)std::min<uint64_t>((c->pool_cap + 255) / 256, 65536)),
                       dim3(256), 0, ctx->stream, c->pool_a, c->pool_b, mark, c->pool_cap, d_old, d_new, n);
    ok = hipGetLastError() == hipSuccess && hipStreamSynchronize(ctx->stream) == hipSuccess;
  }
  (void)hipStreamSynchronize(ctx->stream);
  if (mark) (void)hipFree(mark);
  (void)hipFree(d_old);
  (void)hipFree(d_new);
  if (!ok) {
    am_set_error("am_snapcache_relabel: failed");
    return AM_ERR_HIP;
  }
  return AM_OK;
}

int am_snapcache_destroy(am_snapcache *c) {
  if (!c) return AM_OK;
  if (!c->ctx) return AM_ERR_INVALID;
  AM_LOCK(c->ctx);
  (void)hipSetDevice(c->ctx->device);
  (void)hipStreamSynchronize(c->ctx->stream);
  for (void *p : c->allocs) am_dev_release(c->ctx, p);
  if (c->pool_a) (void)hipFree(c->pool_a);
  if (c->pool_b) (void)hipFree(c->pool_b);
  if (c->pool_p) (void)hipFree(c->pool_p);
  if (c->pool_g) (void)hipFree(c->pool_g);
  delete c;
  return AM_OK;
}

int am_snapcache_read_gc(am_ctx *ctx, am_snapcache *c, const am_op_log *L, const am_read_batch *B,
                         const uint8_t *should_gc, am_read_result *R, uint8_t *gc_mask, uint64_t *thr_vc,
                         uint32_t *thr_pres) {
  if (!ctx || !c || !L || !B || !R || c->ctx != ctx) return AM_ERR_INVALID;
  AM_LOCK(ctx);
  if (L->n_dc != c->n_dc || L->n_keys != c->n_keys) {
    am_set_error("snapshot cache: n_dc / n_keys do not match the log");
    return AM_ERR_INVALID;
  }
  if ((gc_mask || thr_vc || thr_pres) && !(gc_mask && thr_vc && thr_pres)) {
    am_set_error("snapshot cache: gc_mask, thr_vc and thr_pres go together");
    return AM_ERR_INVALID;
  }
  const uint32_t th = B->type_hint;
  if ((th == 0 || th == AM_PN || th == AM_LWW) && !(R->value.v0 && R->value.v1 && R->value.vflag)) {
    am_set_error("snapshot cache reads of PN / LWW keys need value.v0/v1/vflag");
    return AM_ERR_INVALID;
  }
  AM_HIP(hipSetDevice(ctx->device));
  const uint64_t n = B->n_reads;
  if (gc_mask) AM_HIP(hipMemsetAsync(gc_mask, 0, c->n_keys, ctx->stream));
  if (n == 0) return AM_OK;
  const uint32_t nd = c->n_dc;
  // value pool room for every value this batch could store
  uint64_t need = 0, so0 = 0, used = 0;
  if ((th == 0 || th == AM_AWSET || th == AM_MVREG || th == AM_BCOUNTER) && R->value.set_off) {
    void *sz = nullptr;
    if (int rc = am_ctx_scratch(ctx, AM_SCR_SIZES, 64, &sz)) return rc;
    hipLaunchKernelGGL(k_sc_sizes, dim3(1), dim3(64), 0, ctx->stream, R->value.set_off, n, c->ctr, c->wend, c->wend_n,
                       (uint64_t *)sz);
    AM_HIP(hipGetLastError());
    uint64_t w[4] = {0, 0, 0, 0};
    if (int rc = am_ctx_fetch(ctx, sz, 4, w)) return rc;
    c->wend_n = 0;  // consumed: the counter holds them
    need = w[1] - w[0];
    so0 = w[0];
    if (need) {  // this batch's room: one pool word per result word, from `used`
      if (int rc = pool_reserve(c, need, w + 2, &used)) return rc;
    }
  }
  // scratch: code, newest, base_ignore, vflag [n] u8 | base_pres, set_len [n] u32 |
  // base_last_op, v0, v1, set_off [n] u64 | base_vc [nd][n]
  const size_t bytes = n * (4 + 8 + 4 * 8 + (size_t)nd * 8 + 13) + 4096;
  void *scr = nullptr;
  int rc = am_ctx_scratch(ctx, AM_SCR_SNAP, bytes, &scr);
  if (rc) return rc;
  char *p = (char *)scr;
  auto take = [&](size_t b) {
    char *q = p;
    p += (b + 255) & ~(size_t)255;
    return q;
  };
  ScSel S;
  S.base_last_op = (int64_t *)take(n * 8);
  S.v0 = (int64_t *)take(n * 8);
  S.v1 = (uint64_t *)take(n * 8);
  S.set_off = (uint64_t *)take(n * 8);
  S.cp_dst = (uint64_t *)take(n * 8);
  S.cp_len = (uint32_t *)take(n * 4);
  S.base_vc = (uint64_t *)take(n * nd * 8);
  S.base_pres = (uint32_t *)take(n * 4);
  S.set_len = (uint32_t *)take(n * 4);
  S.code = (uint8_t *)take(n);
  S.newest = (uint8_t *)take(n);
  S.base_ignore = (uint8_t *)take(n);
  S.vflag = (uint8_t *)take(n);
  uint8_t *teed = (uint8_t *)take(n);
  const ScView V = view(c);
  hipLaunchKernelGGL(k_sc_claim, dim3(grid(n)), dim3(256), 0, ctx->stream, V, *B);
  hipLaunchKernelGGL(k_sc_select, dim3(grid(n)), dim3(256), 0, ctx->stream, V, *B, S);
  rc = hipGetLastError() == hipSuccess ? AM_OK : AM_ERR_HIP;
  if (rc == AM_OK) {
    am_read_batch db = *B;
    db.base_ignore = S.base_ignore;
    db.base_vc = S.base_vc;
    db.base_pres = S.base_pres;
    db.base_last_op = S.base_last_op;
    db.base = am_values{};
    db.base.v0 = S.v0;
    db.base.v1 = S.v1;
    db.base.vflag = S.vflag;
    db.base.set_off = S.set_off;  // cached pairs: offsets into the pool (set_off[r], set_len[r])
    db.base.set_len = S.set_len;
    db.base.set_a = c->pool_a;
    db.base.set_b = c->pool_b;
    // the group wave kernel tees set pairs into the pool (am_ctx::tee_*)
    const bool tee = need && (th == 0 || th == AM_AWSET || th == AM_MVREG) &&
                     hipMemsetAsync(teed, 0, n, ctx->stream) == hipSuccess;
    ctx->grp_hint_in = c->pool_g;
    if (tee) {
      ctx->tee_a = c->pool_a, ctx->tee_b = c->pool_b, ctx->tee_g = c->pool_g, ctx->tee_done = teed;
      ctx->tee_shift = (int64_t)used - (int64_t)so0;
    }
    rc = am_launch_materialize(ctx, L, &db, R);
    ctx->grp_hint_in = nullptr;
    ctx->tee_a = ctx->tee_b = nullptr, ctx->tee_g = nullptr, ctx->tee_done = nullptr, ctx->tee_shift = 0;
    if (rc == AM_OK) {
      const ScGc G{gc_mask, thr_vc, thr_pres};
      hipLaunchKernelGGL(k_sc_store, dim3(grid(n)), dim3(256), 0, ctx->stream, V, *L, *B, *R, S, should_gc, G, used,
                         so0, need ? c->wend : nullptr, tee ? (const uint8_t *)teed : nullptr);
      if (need) c->wend_n = grid(n) * 4;
      const uint64_t rows = (n + 15) / 16;
      hipLaunchKernelGGL(k_sc_copy, dim3((unsigned)(rows < 65536 ? rows : 65536)), dim3(256), 0, ctx->stream, V, *R, S,
                         n);
      if (hipGetLastError() != hipSuccess) rc = AM_ERR_HIP;
    }
  }
  hipLaunchKernelGGL(k_sc_release, dim3(grid(n)), dim3(256), 0, ctx->stream, V, *B);  // every exit path
  AM_HIP(hipGetLastError());
  return rc;
}

int am_snapcache_read(am_ctx *ctx, am_snapcache *c, const am_op_log *L, const am_read_batch *B, am_read_result *R) {
  return am_snapcache_read_gc(ctx, c, L, B, nullptr, R, nullptr, nullptr, nullptr);
}

int am_snapcache_gc_threshold(am_ctx *ctx, am_snapcache *c, uint8_t *mask, uint64_t *thr_vc, uint32_t *thr_pres) {
  if (!ctx || !c || !mask || !thr_vc || !thr_pres) return AM_ERR_INVALID;
  AM_LOCK(ctx);
  AM_HIP(hipSetDevice(ctx->device));
  if (c->n_keys == 0) return AM_OK;
  hipLaunchKernelGGL(k_sc_threshold, dim3(grid(c->n_keys)), dim3(256), 0, ctx->stream, view(c), mask, thr_vc, thr_pres);
  AM_HIP(hipGetLastError());
  return AM_OK;
}

int am_snapcache_get(am_ctx *ctx, const am_snapcache *c, uint64_t key, uint32_t *n_entries, uint64_t *vc,
                     uint32_t *pres, int64_t *last_op, int64_t *v0, uint64_t *v1, uint8_t *vflag) {
  if (!ctx || !c || !n_entries || key >= c->n_keys) return AM_ERR_INVALID;
  AM_LOCK(ctx);
  AM_HIP(hipSetDevice(ctx->device));
  uint8_t cnt = 0;
  const uint64_t nk = c->n_keys, nd = c->n_dc;
  AM_HIP(hipMemcpyAsync(&cnt, c->cnt + key, 1, hipMemcpyDeviceToHost, ctx->stream));
  // the key's column of each entry-major field (host arrays entry-first: vc [CAP][n_dc])
  if (vc) AM_HIP(hipMemcpy2DAsync(vc, 8, c->vc + key, nk * 8, 8, CAP * nd, hipMemcpyDeviceToHost, ctx->stream));
  if (pres) AM_HIP(hipMemcpy2DAsync(pres, 4, c->pres + key, nk * 4, 4, CAP, hipMemcpyDeviceToHost, ctx->stream));
  if (last_op)
    AM_HIP(hipMemcpy2DAsync(last_op, 8, c->last_op + key, nk * 8, 8, CAP, hipMemcpyDeviceToHost, ctx->stream));
  if (v0) AM_HIP(hipMemcpy2DAsync(v0, 8, c->v0 + key, nk * 8, 8, CAP, hipMemcpyDeviceToHost, ctx->stream));
  if (v1) AM_HIP(hipMemcpy2DAsync(v1, 8, c->v1 + key, nk * 8, 8, CAP, hipMemcpyDeviceToHost, ctx->stream));
  if (vflag) AM_HIP(hipMemcpy2DAsync(vflag, 1, c->vflag + key, nk, 1, CAP, hipMemcpyDeviceToHost, ctx->stream));
  AM_HIP(hipStreamSynchronize(ctx->stream));
  *n_entries = cnt == ABSENT ? AM_SNAPCACHE_ABSENT : cnt;
  return AM_OK;
}

int am_snapcache_get_value(am_ctx *ctx, const am_snapcache *c, uint64_t key, uint32_t e, uint32_t cap_words,
                           uint32_t *n_words, uint64_t *a, uint64_t *b, uint8_t *pres) {
  if (!ctx || !c || !n_words || key >= c->n_keys || e >= CAP) return AM_ERR_INVALID;
  AM_LOCK(ctx);
  AM_HIP(hipSetDevice(ctx->device));
  const uint64_t s = (uint64_t)e * c->n_keys + key;  // entry-major
  uint64_t off = 0;
  uint32_t len = 0;
  AM_HIP(hipMemcpyAsync(&off, c->poff + s, 8, hipMemcpyDeviceToHost, ctx->stream));
  AM_HIP(hipMemcpyAsync(&len, c->plen + s, 4, hipMemcpyDeviceToHost, ctx->stream));
  AM_HIP(hipStreamSynchronize(ctx->stream));
  *n_words = len;
  const uint32_t m = len < cap_words ? len : cap_words;
  if (m && a) AM_HIP(hipMemcpyAsync(a, c->pool_a + off, (size_t)m * 8, hipMemcpyDeviceToHost, ctx->stream));
  if (m && b) AM_HIP(hipMemcpyAsync(b, c->pool_b + off, (size_t)m * 8, hipMemcpyDeviceToHost, ctx->stream));
  if (m && pres) AM_HIP(hipMemcpyAsync(pres, c->pool_p + off, m, hipMemcpyDeviceToHost, ctx->stream));
  AM_HIP(hipStreamSynchronize(ctx->stream));
  return AM_OK;
}

}  // extern "C"
