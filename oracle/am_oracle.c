/*
 * am_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 *
 * Scalar C restatement of the reference's snapshot materialization over the
 * structure-of-arrays op log of include/antidote_mat.h.  It follows the Erlang
 * control flow step by step (paths relative to the reference tree):
 *
 *   amo_materialize_one     clocksi_materializer:materialize/4
 *                           src/clocksi_materializer.erl:89-101
 *     get_first_id          :51-63
 *     walk newest -> oldest materialize_intern / materialize_intern_perform :157-197
 *     is_op_in_snapshot     :216-268 (dict:store / dict:fold / dict:update on the clock)
 *     belongs_to_snapshot_op src/materializer.erl:102-106 (vectorclock:le, hex vectorclock
 *                           0.1.0: union of keys, a missing entry reads 0)
 *     apply_operations      src/clocksi_materializer.erl:113-121, folding Type:update/2
 *                           oldest -> newest; an update that raises gives
 *                           {error, {unexpected_operation, Effect, Type}} (src/materializer.erl:52-58)
 *   amo_gst_min             stable_time_functions:get_min_time/1 (src/stable_time_functions.erl:51-85)
 *   amo_update_stable       meta_data_sender:update_stable/3 (src/meta_data_sender.erl:342-356)
 *
 * CRDT update rules (antidote_crdt @4157110c, un-vendored): PN pinned by the
 * reference's EUnit KATs; LWW = erlang:max(Effect, State) on {Ts, Value} with the
 * initial {0, <<>>}; AW-set = merge of effect entries {Elem, Add, Remove} into the
 * orddict, tokens ToAdd ++ (Current -- Remove), empty elements dropped; MV register
 * = drop overridden tokens then insert_sorted({Value, Token}); bcounter =
 * orddict:update_counter on P[{From,To}] / D[Id].  The last four are parity
 * unpinned (no KAT in the reference).
 *
 * Never linked into the product library.  Built by oracle/Makefile into
 * oracle/_build/libam_oracle.so and loaded by tests/ and bench.py's cpu_baseline.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/antidote_mat.h"

typedef struct {
  uint32_t pres;
  uint64_t t[AM_MAX_DC];
} vc_t;

static uint64_t vc_get(const vc_t *v, unsigned d) { return ((v->pres >> d) & 1u) ? v->t[d] : 0; }

/* vectorclock:le/2 */
static int vc_le(const vc_t *a, const vc_t *b) {
  uint32_t keys = a->pres | b->pres;
  for (unsigned d = 0; d < AM_MAX_DC; ++d)
    if (((keys >> d) & 1u) && !(vc_get(a, d) <= vc_get(b, d))) return 0;
  return 1;
}

static void vc_store(vc_t *v, unsigned d, uint64_t t) {
  v->pres |= 1u << d;
  v->t[d] = t;
}

static uint32_t all_pres(uint32_t n_dc) { return n_dc >= 32 ? 0xFFFFFFFFu : ((1u << n_dc) - 1u); }

static void op_snapshot(const am_op_log *L, uint64_t p, vc_t *out) {
  memset(out, 0, sizeof(*out));
  uint32_t pres = L->snap_pres ? L->snap_pres[p] : all_pres(L->n_dc);
  out->pres = pres & all_pres(L->n_dc);
  const uint64_t stride = L->snap_stride ? L->snap_stride : L->n_ops;
  for (unsigned d = 0; d < L->n_dc; ++d)
    if ((out->pres >> d) & 1u) out->t[d] = L->snap_vc[(uint64_t)d * stride + p];
}

static int64_t op_id_at(const am_op_log *L, uint64_t key, uint64_t p) {
  if (L->op_id) return (int64_t)L->op_id[p];
  uint64_t base = L->key_id_base ? L->key_id_base[key] : 1;
  return (int64_t)(base + (p - L->key_off[key]));
}

/* ---------------- CRDT states ---------------- */
typedef struct {
  uint64_t elem;
  uint64_t *tok;
  uint32_t n, cap;
} aw_ent;

typedef struct {
  aw_ent *e;
  uint32_t n, cap;
} aw_state;

typedef struct {
  uint64_t val, tok;
} mv_pair;

typedef struct {
  mv_pair *p;
  uint32_t n, cap;
} mv_state;

static void *xrealloc(void *p, size_t n) {
  void *q = realloc(p, n ? n : 1);
  if (!q) abort();
  return q;
}

static void aw_push_tok(aw_ent *e, uint64_t t) {
  if (e->n == e->cap) {
    e->cap = e->cap ? 2 * e->cap : 4;
    e->tok = (uint64_t *)xrealloc(e->tok, e->cap * sizeof(uint64_t));
  }
  e->tok[e->n++] = t;
}

static void aw_free(aw_state *s) {
  for (uint32_t i = 0; i < s->n; ++i) free(s->e[i].tok);
  free(s->e);
  memset(s, 0, sizeof(*s));
}

static int contains(const uint64_t *a, uint64_t n, uint64_t x) {
  for (uint64_t i = 0; i < n; ++i)
    if (a[i] == x) return 1;
  return 0;
}

/* Current -- ToRemove (lists:subtract/2): each token of rm removes the first occurrence
 * of that token from cur; the order of cur is kept.  Appends the result to ne. */
static void aw_push_subtract(aw_ent *ne, const uint64_t *cur, uint32_t ncur, const uint64_t *rm, uint64_t nr) {
  uint8_t *gone = (uint8_t *)calloc(ncur ? ncur : 1, 1);
  for (uint64_t j = 0; j < nr; ++j)
    for (uint32_t i = 0; i < ncur; ++i)
      if (!gone[i] && cur[i] == rm[j]) {
        gone[i] = 1;
        break;
      }
  for (uint32_t i = 0; i < ncur; ++i)
    if (!gone[i]) aw_push_tok(ne, cur[i]);
  free(gone);
}

/* antidote_crdt_set_aw:update/2 -- apply_downstreams merge.  Returns 0, or -1 on a malformed effect. */
static int aw_apply(aw_state *s, const uint64_t *eff, uint64_t len) {
  aw_state out = {0};
  uint64_t q = 0;
  uint32_t si = 0;
  /* parse entries lazily: each [elem, n_add, n_rm, add..., rm...] */
  for (;;) {
    int have_op = q < len;
    uint64_t e1 = 0, na = 0, nr = 0;
    const uint64_t *add = 0, *rm = 0;
    if (have_op) {
      if (q + 3 > len) goto bad;
      e1 = eff[q];
      na = eff[q + 1];
      nr = eff[q + 2];
      if (na > len || nr > len || q + 3 + na + nr > len) goto bad;
      add = eff + q + 3;
      rm = add + na;
    }
    int have_set = si < s->n;
    if (!have_op && !have_set) break;
    aw_ent ne = {0};
    if (have_op && (!have_set || e1 < s->e[si].elem)) {
      /* element not in the state: [{Elem1, ToAdd}] if ToAdd /= [] */
      ne.elem = e1;
      for (uint64_t i = 0; i < na; ++i) aw_push_tok(&ne, add[i]);
      q += 3 + na + nr;
    } else if (have_op && e1 == s->e[si].elem) {
      ne.elem = e1;
      for (uint64_t i = 0; i < na; ++i) aw_push_tok(&ne, add[i]);  /* ToAdd ++ (Current -- ToRemove) */
      aw_push_subtract(&ne, s->e[si].tok, s->e[si].n, rm, nr);
      q += 3 + na + nr;
      ++si;
    } else {
      ne.elem = s->e[si].elem;
      for (uint32_t i = 0; i < s->e[si].n; ++i) aw_push_tok(&ne, s->e[si].tok[i]);
      ++si;
    }
    if (ne.n == 0) {
      free(ne.tok);
      continue;
    }
    if (out.n == out.cap) {
      out.cap = out.cap ? 2 * out.cap : 8;
      out.e = (aw_ent *)xrealloc(out.e, out.cap * sizeof(aw_ent));
    }
    out.e[out.n++] = ne;
  }
  aw_free(s);
  *s = out;
  return 0;
bad:
  aw_free(&out);
  return -1;
}

static int mv_cmp(const mv_pair *a, const mv_pair *b) {
  if (a->val != b->val) return a->val < b->val ? -1 : 1;
  if (a->tok != b->tok) return a->tok < b->tok ? -1 : 1;
  return 0;
}

/* antidote_crdt_register_mv:update/2 */
static void mv_apply(mv_state *s, int reset, uint64_t val, uint64_t tok, const uint64_t *ovr, uint64_t no) {
  uint32_t w = 0;
  for (uint32_t i = 0; i < s->n; ++i)
    if (!contains(ovr, no, s->p[i].tok)) s->p[w++] = s->p[i];
  s->n = w;
  if (reset) return;
  mv_pair a = {val, tok};
  uint32_t pos = 0;
  while (pos < s->n && mv_cmp(&a, &s->p[pos]) > 0) ++pos;
  if (pos < s->n && mv_cmp(&a, &s->p[pos]) == 0) return;
  if (s->n == s->cap) {
    s->cap = s->cap ? 2 * s->cap : 8;
    s->p = (mv_pair *)xrealloc(s->p, s->cap * sizeof(mv_pair));
  }
  memmove(s->p + pos + 1, s->p + pos, (s->n - pos) * sizeof(mv_pair));
  s->p[pos] = a;
  s->n++;
}

static int add_ovf(__int128 *acc, __int128 v) {
  *acc += v;
  return 0;
}

/* ---------------- materialize/4 ---------------- */
int amo_materialize_one(const am_op_log *L, const am_read_batch *B, uint64_t r, am_read_result *R) {
  const uint32_t nd = L->n_dc;
  const uint64_t n = B->n_reads;
  const uint64_t key = B->key[r];
  const unsigned type = B->type[r];
  vc_t S = {0}, C0 = {0}, last_ct = {0};
  const uint64_t *rv = B->read_vc;
  const uint64_t rstride = B->per_read_clock ? n : 1, ridx = B->per_read_clock ? r : 0;
  S.pres = B->read_pres[ridx] & all_pres(nd);
  for (unsigned d = 0; d < nd; ++d) S.t[d] = rv[(uint64_t)d * rstride + ridx];
  const int has_txid = B->txid && (!B->txid_valid || B->txid_valid[r]);
  const uint64_t txid = has_txid ? B->txid[r] : 0;
  const int base_ignore = !B->base_ignore || B->base_ignore[r];
  if (!base_ignore) {
    C0.pres = B->base_pres[r] & all_pres(nd);
    for (unsigned d = 0; d < nd; ++d) C0.t[d] = B->base_vc[(uint64_t)d * n + r];
  }
  const uint64_t off0 = L->key_off[key], off1 = L->key_off[key + 1];
  const uint64_t nops = off1 - off0;

  int32_t status = AM_OK;
  uint8_t flags = 0;
  /* get_first_id/1 */
  int64_t first_hole = nops == 0 ? 0 : op_id_at(L, key, off1 - 1);
  int last_ignore = base_ignore;
  if (!base_ignore) last_ct = C0;
  int new_ss = 0;
  uint64_t *incl = (uint64_t *)malloc((nops ? nops : 1) * sizeof(uint64_t));
  uint64_t n_incl = 0;

  /* materialize_intern: newest -> oldest */
  for (uint64_t k = 0; k < nops; ++k) {
    const uint64_t p = off1 - 1 - k;
    if (L->key_type[key] != type || (L->key_flags && (L->key_flags[key] & AM_KEY_MIXED_TYPES))) {
      status = AM_ERR_CORRUPTED_OPS_CACHE;
      break;
    }
    const unsigned dc = AM_META_DC(L->op_meta[p]);
    const uint64_t ct = L->commit_time[p];
    vc_t opss;
    op_snapshot(L, p, &opss);
    /* is_op_in_snapshot/7 */
    vc_t opss1 = opss;
    vc_store(&opss1, dc, ct);
    int belongs = base_ignore ? 1 : !vc_le(&opss1, &C0);
    int txmatch = has_txid && L->op_txid && L->op_txid[p] == txid;
    if (belongs || txmatch) {
      vc_t newtime = last_ignore ? opss1 : last_ct;
      int acc = 1;
      for (unsigned d = 0; d < AM_MAX_DC; ++d) {
        if (!((opss1.pres >> d) & 1u)) continue;
        const uint64_t time_op = opss1.t[d];
        int res1;
        if ((S.pres >> d) & 1u)
          res1 = (S.t[d] < time_op) ? 0 : acc;
        else {
          flags |= AM_FLAG_MISSING_DC_LOGGED;
          res1 = 0;
        }
        if ((newtime.pres >> d) & 1u)
          newtime.t[d] = time_op > newtime.t[d] ? time_op : newtime.t[d];
        else
          vc_store(&newtime, d, time_op);
        acc = res1;
      }
      if (acc) {
        incl[n_incl++] = p;
        last_ct = newtime;
        last_ignore = 0;
        new_ss = 1;
      } else {
        first_hole = op_id_at(L, key, p) - 1;
      }
    }
  }

  uint32_t count = 0;
  if (status == AM_OK) {
    /* apply_operations: oldest -> newest (incl[] holds newest first) */
    const am_values *bv = &B->base;
    am_values *ov = &R->value;
    if (type == AM_PN) {
      __int128 acc = (bv->v0) ? (__int128)bv->v0[r] : 0;
      for (uint64_t j = n_incl; j-- > 0;) {
        const uint64_t p = incl[j];
        if (L->op_meta[p] & AM_META_BAD) {
          status = AM_ERR_UNEXPECTED_OPERATION;
          break;
        }
        add_ovf(&acc, (__int128)(int64_t)L->p0[p]);
        ++count;
      }
      if (status == AM_OK && (acc > (__int128)INT64_MAX || acc < (__int128)INT64_MIN)) status = AM_ERR_OVERFLOW;
      if (status == AM_OK) ov->v0[r] = (int64_t)acc;
    } else if (type == AM_LWW) {
      uint64_t ts = bv->v0 ? (uint64_t)bv->v0[r] : 0;
      uint64_t val = bv->v1 ? bv->v1[r] : 0;
      uint8_t isbin = bv->vflag ? bv->vflag[r] : 1;
      if (!bv->v0) isbin = 1;
      for (uint64_t j = n_incl; j-- > 0;) {
        const uint64_t p = incl[j];
        if (L->op_meta[p] & AM_META_BAD) {
          status = AM_ERR_UNEXPECTED_OPERATION;
          break;
        }
        /* erlang:max({Ts, Val}, State): the effect replaces the state iff it is larger */
        const uint64_t ets = L->p0[p], eval = L->p1[p];
        int gt;
        if (ets != ts)
          gt = ets > ts;
        else if (isbin)
          gt = 0; /* a binary sorts above every integer */
        else
          gt = eval > val;
        if (gt) {
          ts = ets;
          val = eval;
          isbin = 0;
        }
        ++count;
      }
      if (status == AM_OK) {
        ov->v0[r] = (int64_t)ts;
        ov->v1[r] = val;
        ov->vflag[r] = isbin;
      }
    } else if (type == AM_AWSET) {
      aw_state st = {0};
      if (bv->set_off) { /* base pairs (elem, token): the orddict in state order */
        for (uint64_t i = bv->set_off[r]; i < bv->set_off[r] + bv->set_len[r]; ++i) {
          if (st.n == 0 || st.e[st.n - 1].elem != bv->set_a[i]) {
            if (st.n == st.cap) {
              st.cap = st.cap ? 2 * st.cap : 8;
              st.e = (aw_ent *)xrealloc(st.e, st.cap * sizeof(aw_ent));
            }
            memset(&st.e[st.n], 0, sizeof(aw_ent));
            st.e[st.n++].elem = bv->set_a[i];
          }
          aw_push_tok(&st.e[st.n - 1], bv->set_b[i]);
        }
      }
      for (uint64_t j = n_incl; j-- > 0;) {
        const uint64_t p = incl[j];
        const uint64_t *eff = L->var_off ? L->var_data + L->var_off[p] : 0;
        const uint64_t elen = L->var_off ? L->var_off[p + 1] - L->var_off[p] : 0;
        if ((L->op_meta[p] & AM_META_BAD) || aw_apply(&st, eff, elen) != 0) {
          status = AM_ERR_UNEXPECTED_OPERATION;
          break;
        }
        ++count;
      }
      if (status == AM_OK) {
        uint64_t o = ov->set_off[r], cap = ov->set_off[r + 1] - o, w = 0;
        for (uint32_t i = 0; i < st.n && status == AM_OK; ++i) {
          for (uint32_t t = 0; t < st.e[i].n; ++t) { /* the token list in state order */
            if (w >= cap) {
              status = AM_ERR_CAPACITY;
              break;
            }
            ov->set_a[o + w] = st.e[i].elem;
            ov->set_b[o + w] = st.e[i].tok[t];
            ++w;
          }
        }
        if (status == AM_OK) ov->set_len[r] = (uint32_t)w;
      }
      aw_free(&st);
    } else if (type == AM_MVREG) {
      mv_state st = {0};
      if (bv->set_off) {
        for (uint64_t i = bv->set_off[r]; i < bv->set_off[r] + bv->set_len[r]; ++i) {
          if (st.n == st.cap) {
            st.cap = st.cap ? 2 * st.cap : 8;
            st.p = (mv_pair *)xrealloc(st.p, st.cap * sizeof(mv_pair));
          }
          st.p[st.n].val = bv->set_a[i];
          st.p[st.n].tok = bv->set_b[i];
          st.n++;
        }
      }
      for (uint64_t j = n_incl; j-- > 0;) {
        const uint64_t p = incl[j];
        if (L->op_meta[p] & AM_META_BAD) {
          status = AM_ERR_UNEXPECTED_OPERATION;
          break;
        }
        const int reset = AM_META_KIND(L->op_meta[p]) == AM_MV_RESET;
        const uint64_t *ovr = L->var_off ? L->var_data + L->var_off[p] : 0;
        const uint64_t no = L->var_off ? L->var_off[p + 1] - L->var_off[p] : 0;
        mv_apply(&st, reset, L->p0[p], L->p1[p], ovr, no);
        ++count;
      }
      if (status == AM_OK) {
        uint64_t o = ov->set_off[r], cap = ov->set_off[r + 1] - o;
        if (st.n > cap)
          status = AM_ERR_CAPACITY;
        else {
          for (uint32_t i = 0; i < st.n; ++i) {
            ov->set_a[o + i] = st.p[i].val;
            ov->set_b[o + i] = st.p[i].tok;
          }
          ov->set_len[r] = st.n;
        }
      }
      free(st.p);
    } else if (type == AM_BCOUNTER) {
      const uint32_t np = nd * nd;
      __int128 pv[AM_MAX_DC * AM_MAX_DC];
      uint8_t pp[AM_MAX_DC * AM_MAX_DC];
      __int128 dv[AM_MAX_DC];
      uint8_t dp[AM_MAX_DC];
      memset(pv, 0, sizeof(pv)), memset(pp, 0, sizeof(pp)), memset(dv, 0, sizeof(dv)), memset(dp, 0, sizeof(dp));
      if (bv->set_off && bv->set_len)  /* the base orddicts: (slot, value) entries */
        for (uint32_t i = 0; i < bv->set_len[r]; ++i) {
          const uint64_t slot = bv->set_a[bv->set_off[r] + i];
          const int64_t v = (int64_t)bv->set_b[bv->set_off[r] + i];
          if (slot < np) pv[slot] = v, pp[slot] = 1;
          else if (slot < np + nd) dv[slot - np] = v, dp[slot - np] = 1;
        }
      for (uint64_t j = n_incl; j-- > 0;) {
        const uint64_t p = incl[j];
        const unsigned kind = AM_META_KIND(L->op_meta[p]);
        const unsigned from = (unsigned)(L->p1[p] & 0xFF), to = (unsigned)((L->p1[p] >> 8) & 0xFF);
        if ((L->op_meta[p] & AM_META_BAD) || kind > AM_BC_TRANSFER || from >= nd || to >= nd) {
          status = AM_ERR_UNEXPECTED_OPERATION;
          break;
        }
        const int64_t v = (int64_t)L->p0[p];
        if (kind == AM_BC_INCREMENT) {
          pv[from * nd + from] += v;
          pp[from * nd + from] = 1;
        } else if (kind == AM_BC_DECREMENT) {
          dv[from] += v;
          dp[from] = 1;
        } else {
          pv[from * nd + to] += v;
          pp[from * nd + to] = 1;
        }
        ++count;
      }
      if (status == AM_OK) {
        for (uint32_t i = 0; i < np; ++i)
          if (pv[i] > (__int128)INT64_MAX || pv[i] < (__int128)INT64_MIN) status = AM_ERR_OVERFLOW;
        for (uint32_t i = 0; i < nd; ++i)
          if (dv[i] > (__int128)INT64_MAX || dv[i] < (__int128)INT64_MIN) status = AM_ERR_OVERFLOW;
      }
      if (status == AM_OK) {  /* the touched entries, P then D, each in key order */
        const uint64_t o = ov->set_off[r], cap = ov->set_off[r + 1] - o;
        uint32_t ne = 0;
        for (uint32_t i = 0; i < np + nd; ++i) {
          const int present = i < np ? pp[i] : dp[i - np];
          if (!present) continue;
          if (ne < cap) {
            ov->set_a[o + ne] = i;
            ov->set_b[o + ne] = (uint64_t)(int64_t)(i < np ? pv[i] : dv[i - np]);
          }
          ++ne;
        }
        if (ne > cap) status = AM_ERR_CAPACITY;
        else ov->set_len[r] = ne;
      }
    } else {
      status = AM_ERR_UNEXPECTED_OPERATION;
    }
  }
  free(incl);

  R->status[r] = status;
  R->flags[r] = flags;
  if (status == AM_OK) {
    R->new_last_op[r] = first_hole;
    R->last_ct_ignore[r] = (uint8_t)last_ignore;
    R->last_ct_pres[r] = last_ignore ? 0 : last_ct.pres;
    for (unsigned d = 0; d < nd; ++d)
      R->last_ct[(uint64_t)d * n + r] = (!last_ignore && ((last_ct.pres >> d) & 1u)) ? last_ct.t[d] : 0;
    R->is_new_ss[r] = (uint8_t)new_ss;
    R->count[r] = count;
  }
  return status;
}

/* Materialize reads [r0, r1).  Thread-safe (no shared state). */
int amo_materialize_range(const am_op_log *L, const am_read_batch *B, uint64_t r0, uint64_t r1,
                          am_read_result *R) {
  for (uint64_t r = r0; r < r1; ++r) amo_materialize_one(L, B, r, R);
  return 0;
}

/* stable_time_functions:get_min_time/1 over n_part partition clocks (partition-major
 * [n_part][n_dc]); undef[p] != 0 marks an 'undefined' partition. */
int amo_gst_min(uint32_t n_dc, uint32_t n_part, const uint64_t *vc, const uint32_t *pres, const uint8_t *undef,
                uint64_t *out_vc, uint32_t *out_pres) {
  uint32_t mp = 0;
  int found_undef = 0;
  for (unsigned d = 0; d < n_dc; ++d) out_vc[d] = 0;
  for (uint32_t p = 0; p < n_part; ++p) {
    if (undef && undef[p]) {
      found_undef = 1;
      continue;
    }
    for (unsigned d = 0; d < n_dc; ++d) {
      if (!((pres[p] >> d) & 1u)) continue;
      const uint64_t t = vc[(uint64_t)p * n_dc + d];
      const uint64_t prev = ((mp >> d) & 1u) ? out_vc[d] : t;
      out_vc[d] = prev >= t ? t : prev;
      mp |= 1u << d;
    }
  }
  if (found_undef)
    for (unsigned d = 0; d < n_dc; ++d)
      if ((mp >> d) & 1u) out_vc[d] = 0;
  *out_pres = mp;
  return 0;
}

/* meta_data_sender:update_stable/3 with update_func_min/2; returns the Bool. */
int amo_update_stable(uint32_t n_dc, uint64_t *last_vc, uint32_t *last_pres, const uint64_t *new_vc,
                      uint32_t new_pres) {
  int changed = 0;
  for (unsigned d = 0; d < n_dc; ++d) {
    if (!((new_pres >> d) & 1u)) continue;
    if (!((*last_pres >> d) & 1u) || new_vc[d] >= last_vc[d]) {
      last_vc[d] = new_vc[d];
      *last_pres |= 1u << d;
      changed = 1;
    }
  }
  return changed;
}
