/*
 * antidote_mat.h -- C ABI of the MI355X batched CRDT snapshot materializer.
 *
 * Drop-in boundary for the AntidoteDB Cure/ClockSI snapshot-read hot path.
 * Every entry point names the reference interface it replaces (paths are
 * relative to the reference tree, SmallEndian/antidote):
 *
 *   am_materialize          clocksi_materializer:materialize/4
 *                           (src/clocksi_materializer.erl:82-101), batched over keys;
 *                           called from materializer_vnode:materialize_snapshot/7
 *                           (src/materializer_vnode.erl:469-509, call at :478)
 *   am_store_create         the per-partition ETS ops cache laid out in HBM
 *                           (materializer_vnode:op_insert_gc/3 appends,
 *                           src/materializer_vnode.erl:622-647; tuple layout
 *                           include/antidote.hrl:81-90)
 *   am_gst_local_min        stable_time_functions:get_min_time/1 over the local
 *                           partitions (src/stable_time_functions.erl:51-85)
 *   am_gst_allreduce        the node-to-node broadcast + merge of meta_data_sender
 *                           (src/meta_data_sender.erl:232-255) as one RCCL min
 *                           all-reduce over xGMI
 *   am_gst_finalize         meta_data_sender:update_stable/3 with
 *                           stable_time_functions:update_func_min/2
 *                           (src/meta_data_sender.erl:342-356,
 *                           src/stable_time_functions.erl:42-48) and the gr-mode
 *                           broadcast of dc_utilities:get_stable_snapshot/0
 *                           (src/dc_utilities.erl:246-279)
 *   am_snapcache_read       materializer_vnode:internal_read/7 with the snapshot cache
 *                           in HBM: get_from_snapshot_cache/5, vector_orddict:
 *                           get_smaller/2 + insert_bigger/3, materialize_snapshot/7,
 *                           internal_store_ss/4 (src/materializer_vnode.erl:342-509,
 *                           src/vector_orddict.erl:75-140)
 *   am_store_update         op-cache ingestion + GC: materializer_vnode:op_insert_gc/3
 *                           appends (src/materializer_vnode.erl:622-647) and prune_ops/2
 *                           + check_filter/7 (:565-604) as one batched log rebuild
 *   am_snapcache_gc_threshold  the prune threshold of snapshot_insert_gc/4 (:515-535):
 *                           vectorclock:min over the first SNAPSHOT_MIN cached snapshots
 *   am_vnode_insert_host    one partition's materializer_vnode state: op_insert_gc/3 with
 *   am_vnode_read_host      its write-triggered GC read (src/materializer_vnode.erl:622-647),
 *                           internal_read/7 with ShouldGC (:371-376), load_ops/2 (:312-319)
 *   am_read_objects_submit  clocksi_interactive_coord's read_objects fan-out over a GPU's
 *                           partitions (src/clocksi_interactive_coord.erl:732-747,
 *                           src/clocksi_readitem_server.erl:217-228) as one async batch
 *   am_key_partition        log_utilities:get_key_partition/1 + convert_key/1: integer
 *   am_key_partition_bytes  keys, binaries (list_to_integer text or SHA-1 chash_key) and
 *                           other terms (src/log_utilities.erl:60-79,100-118)
 *   am_codec_*              Erlang terms of CRDT states <-> order-preserving u64 labels
 *                           (the NIF's term conversion)
 *
 * Conventions
 *   - Plain C, POD structure-of-arrays, no framework types.  Status codes
 *     mirror the reference's error conventions: {error, {unexpected_operation,
 *     Effect, Type}} (src/materializer.erl:52-58) and
 *     erlang:error(corrupted_ops_cache) (src/clocksi_materializer.erl:190-191).
 *   - A vectorclock (a dict DcId -> time in the reference, hex vectorclock 0.1.0)
 *     is a dense array of n_dc u64 lanes plus a presence bitmask (bit d set =
 *     DC d is a key of the dict).  DC ids are mapped by the caller to indices
 *     0..n_dc-1 in ascending Erlang term order (so sorted [{Dc, T}] renderings
 *     match).  n_dc <= AM_MAX_DC.
 *   - "ignore" (an atom in the reference) is an explicit flag.
 *   - Device entry points take DEVICE pointers and run on the context's HIP
 *     stream, asynchronously but for the data-dependent counter readbacks each
 *     one documents (am_materialize: at most two); the *_host variants take host
 *     memory and block.
 */
#ifndef ANTIDOTE_MAT_H
#define ANTIDOTE_MAT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AM_ABI_VERSION 12
#define AM_MAX_DC 32

/* CRDT types (the reference's type atoms) */
enum am_type {
  AM_PN = 1,        /* antidote_crdt_counter_pn   */
  AM_LWW = 2,       /* antidote_crdt_register_lww */
  AM_AWSET = 3,     /* antidote_crdt_set_aw       */
  AM_MVREG = 4,     /* antidote_crdt_register_mv  */
  AM_BCOUNTER = 5   /* antidote_crdt_counter_b    */
};

/* Per-read status.  >0: the reference's {error, _} / exception outcomes. <0: API errors. */
enum am_status {
  AM_OK = 0,
  AM_ERR_CORRUPTED_OPS_CACHE = 1,   /* erlang:error(corrupted_ops_cache)            */
  AM_ERR_UNEXPECTED_OPERATION = 2,  /* {error, {unexpected_operation, Effect, Type}}*/
  AM_ERR_OVERFLOW = 3,              /* result outside int64 (Erlang would bignum)   */
  AM_ERR_CAPACITY = 4,              /* set result larger than the caller's capacity */
  AM_ERR_COLD_PATH = 5,             /* no cached snapshot at or below the read clock:
                                       get_from_snapshot_log (the log, not the cache) */
  AM_ERR_INVALID = -1,
  AM_ERR_HIP = -2,
  AM_ERR_RCCL = -3,
  AM_ERR_NOMEM = -4,
  AM_ERR_UNSUPPORTED = -5
};

/* per-read informational flags */
#define AM_FLAG_MISSING_DC_LOGGED 0x1u  /* logger:error("Could not find DC in SS"), src/clocksi_materializer.erl:246 */

/* op_meta byte: commit DC index, effect sub-kind, invalid-effect marker */
#define AM_META_DC(m) ((unsigned)(m)&0x1Fu)
#define AM_META_KIND(m) (((unsigned)(m) >> 5) & 0x3u)
#define AM_META_BAD 0x80u /* Type:update/2 raises on this effect */
#define AM_MAKE_META(dc, kind, bad) ((uint8_t)(((dc)&0x1F) | (((kind)&3) << 5) | ((bad) ? 0x80 : 0)))

/* effect sub-kinds */
#define AM_MV_ASSIGN 0 /* {Value, Token, Overridden}  */
#define AM_MV_RESET 1  /* {reset, Overridden}         */
#define AM_BC_INCREMENT 0 /* {{increment, V}, Id}      -> P[{Id,Id}] += V   */
#define AM_BC_DECREMENT 1 /* {{decrement, V}, Id}      -> D[Id] += V        */
#define AM_BC_TRANSFER 2  /* {{transfer, V, To}, From} -> P[{From,To}] += V */

/* key_flags */
#define AM_KEY_MIXED_TYPES 0x1u /* the key's log holds ops of more than one type */

/*
 * The per-partition ops cache as structure-of-arrays (one "log" = one
 * materializer_vnode ops_cache table).  Ops of key k occupy
 * [key_off[k], key_off[k+1]) oldest -> newest, exactly the ETS tuple order
 * (slot FIRST_OP .. FIRST_OP+Length-1).  Payload encoding per type:
 *   PN        p0 = int64 delta
 *   LWW       p0 = timestamp, p1 = value (u64)
 *   MVREG     p0 = value, p1 = token, var = overridden tokens (kind ASSIGN|RESET)
 *   AWSET     var = entries [elem, n_add, n_rm, add_tok..., rm_tok...]...,
 *             entries sorted by elem, elems unique within one effect
 *   BCOUNTER  p0 = int64 amount, p1 = from | (to << 8), kind in op_meta
 */
typedef struct am_op_log {
  uint32_t n_dc;
  uint32_t _pad;
  uint64_t n_keys;
  uint64_t n_ops;
  uint64_t n_var;
  uint64_t snap_stride;        /* elements between the DC columns of snap_vc; 0 => n_ops */
  const uint64_t *key_off;     /* [n_keys+1]                                        */
  const uint64_t *key_id_base; /* [n_keys] op id of the key's oldest op; NULL => 1   */
  const uint8_t *key_type;     /* [n_keys] am_type                                   */
  const uint8_t *key_flags;    /* [n_keys] or NULL                                   */
  const uint8_t *op_meta;      /* [n_ops]                                            */
  const uint64_t *commit_time; /* [n_ops] commit_time = {DcId, CT}: the CT           */
  const uint64_t *snap_vc;     /* [n_dc][snap_stride] snapshot_time, DC-major        */
  const uint32_t *snap_pres;   /* [n_ops] presence of snapshot_time keys; NULL=all   */
  const uint64_t *op_txid;     /* [n_ops] or NULL (never equal to a read's TxId)     */
  const uint64_t *op_id;       /* [n_ops] or NULL (dense ids from key_id_base)       */
  const uint64_t *p0;          /* [n_ops]                                            */
  const uint64_t *p1;          /* [n_ops]                                            */
  const uint64_t *var_off;     /* [n_ops+1] or NULL                                  */
  const uint64_t *var_data;    /* [n_var]                                            */
  /* Packed streaming view (logs without snap_pres), built on the device by am_store_create /
   * am_store_update / am_synth_store (NULL in host logs).  The op's commit vector
   * X = snapshot_time with X[dc] = commit_time (the clock is_op_in_snapshot/7 compares) is
   * stored relative to a per-key time base:
   *   pk_vc[d][p] = X[d] - key_tbase[k]   as u32 in [0, 2^32 - 2]
   * key_tbase[k] = (the smallest entry of the key's first op that lies within 2^31 of its
   * commit time) - 2^30, saturating at 0.  An op with an entry outside the window, or
   * carrying AM_META_BAD, has pk_vc[0][p] = AM_PK_ESC and is read from the full columns
   * above.  The inclusion test then runs on u32 (one compare and one max per DC) and
   * streams 4 * n_dc bytes per op: 32 B at D = 8 instead of 72 B. */
  const uint64_t *key_tbase;   /* [n_keys]                                           */
  const uint32_t *pk_vc;       /* [n_dc][snap_stride]                                */
  /* Token-group view (add-wins set and MV register keys), built on the device with the
   * packed view (am_store_create / am_store_update / am_synth_store).  Every effect is
   * flattened to births and kills of tokens:
   *   AW  add token t of elem e -> birth of (e, t);  remove token t of elem e -> kill of (e, t)
   *   MV  {Value, Token, _}      -> birth of (Value, Token); overridden token t -> kill of t
   * A key's distinct kill keys (AW (elem, token), MV token) are its GROUPS, numbered in the
   * reference's output order: AW by elem, then newest birth first (ToAdd ++ Current), MV by
   * (Value, Token) (insert_sorted); groups without a birth last.  One u32 record per
   * birth / EFFECTIVE kill (one that follows its group's birth: a kill in the birth's own op
   * or earlier never removes the token; every kill of a group with no birth in the log, whose
   * token only a cached base can hold), a key's records contiguous and in op order,
   * [rec_key_off[k], rec_key_off[k+1]):
   *   rec_g = op index within the key (bits 0-15) | kill << 16 | group << 17, or 0xFFFFFFFF
   *           for a kill slot that is not effective
   * and group g of key k is the pair grp[2 (rec_key_off[k] + g) + {0, 1}] (AW (elem, token), MV
   * (Value, Token); MV groups without a birth (~0, token)).  key_ngrp[k] = number of groups,
   * or AM_NGRP_NONE when the key is materialized from var_data instead (more than
   * AM_GRP_MAX_REC records or 2^16 ops, or a log outside the closed form: a token born
   * twice).  A materialization then streams the ops (inclusion), the records (born / killed
   * bits per group) and only the surviving groups' pairs, with no sort.  Ops carrying
   * AM_META_BAD produce no record; an op whose variable payload is malformed (Type:update/2
   * would raise) gets AM_META_BAD set in op_meta and is escaped in the packed view. */
  uint64_t n_rec;
  const uint64_t *rec_key_off; /* [n_keys+1]                                         */
  const uint32_t *rec_g;       /* [n_rec]                                            */
  const uint64_t *grp;         /* [n_rec][2], 16-byte aligned: one load per survivor */
  const uint32_t *key_ngrp;    /* [n_keys]                                           */
  /* Room for appends (the ETS tuple's ListLen slack, src/materializer_vnode.erl:540-560; vnode
   * stores only, NULL elsewhere).  With key_end set, key k's ops are [key_off[k], key_end[k])
   * and [key_end[k], key_off[k+1]) is free room that am_store_apply fills in place (always at
   * least one free slot: var_off[key_end[k]] ends the key's last op's words); with rec_key_end
   * set, its records are [rec_key_off[k], rec_key_end[k]) with room up to rec_key_off[k+1]
   * (group g still at grp[2 (rec_key_off[k] + g)]).  Every reader takes a key's end from
   * key_end when present, else key_off[k+1]. */
  const uint64_t *key_end;     /* [n_keys] or NULL                                   */
  const uint64_t *rec_key_end; /* [n_keys] or NULL                                   */
  /* Group-mask view (built with the token-group view): for the ops of a grouped key with at
   * most 32 groups, gmask[p] = the groups op p births (bits 0-31) | the groups it EFFECTIVELY
   * kills (bits 32-63) -- the key's records folded per op, so a short read ORs one word per
   * included op instead of testing records; 0 for every other op.  NULL in host logs. */
  const uint64_t *gmask;       /* [n_ops] or NULL                                    */
  /* Zone map (device stores, NULL in host logs): per block z of AM_ZONE_OPS consecutive op
   * slots [z * AM_ZONE_OPS, (z + 1) * AM_ZONE_OPS) of the columns, zone_vc[d * n_zones + z] >=
   * X[d] of every op in the block (X = the commit vector is_op_in_snapshot/7 compares;
   * n_zones = ceil(snap_stride or n_ops / AM_ZONE_OPS)).  An upper bound, kept by every writer
   * (a GC may leave it above the surviving ops).  A read with a base snapshot skips a block
   * whose bound is vectorclock:le the base clock: none of its ops is a candidate
   * (belongs_to_snapshot_op/3), so none counts, none is applied and none bounds NewLastOp --
   * the ops already folded into the cached snapshot are not streamed again.
   * Row n_dc, zone_vc[n_dc * n_zones + z] = 1 marks an EXACT block: all its slots are used ops
   * of one key, none escaped from the packed view or invalid, and the bound is their maximum.
   * A read whose clock covers an exact block's bound includes every op of it: its inclusion
   * bits, count and LastOpCt maxima come from the mark and the bound, without the ops' commit
   * vectors.
   * Rows n_dc + 1 .. n_dc + 3 (zone_gsum non-NULL): an exact block of a grouped add-wins-set /
   * MV-register key with at most AM_GRP_MAX_REC groups has its group summary at word
   * zone_vc[(n_dc + 1) * n_zones + z] of zone_gsum (else ~0 -- rows n_dc + 2 and n_dc + 3 are
   * then meaningless), its records end (exclusive, a rec_g index) at row n_dc + 2 and its records
   * begin at row n_dc + 3.  Row n_dc + 4 is the block's summary slot, (capacity in words << 48) |
   * word offset, or 0: a block inside a grouped key's op range (room included) owns one, so
   * am_store_apply can rewrite the summary in place when the block becomes exact again.
   * Maintenance: am_store_apply recomputes, for every block inside a key it writes (room
   * included), the exact maxima over the used slots, the mark, and the summary when the key's
   * new group count fits the slot (else row n_dc + 1 = ~0); a block shared with another key only
   * has its bound raised.  am_store_index drops or (re)builds the whole index. */
  const uint64_t *zone_vc;
  /* Zone group summaries (device stores, or NULL): for such a block, ceil(G/32) born words then
   * ceil(G/32) killed words over the key's G groups -- the OR of its ops' token-group records,
   * so a read including the whole block sets those bits without streaming its records. */
  const uint32_t *zone_gsum;
  /* Birth-ordered pairs (device stores with the token-group view, or NULL): for a birth
   * record rec_g[i] of a grouped key, prec[2 i + {0, 1}] = its group's pair (grp above); other
   * slots unspecified.  Records are in op order, so the groups that survive a read -- in an
   * add-wins set the newest add of each element, in an MV register the newest assigns --
   * have their births close together here, while in grp (output order) they lie a group run
   * apart: the record pass gathers a survivor's pair through its birth record. */
  const uint64_t *prec;        /* [n_rec][2] or NULL                                 */
  /* Escape rows (device stores with the packed view and n_dc >= 2, or NULL): an op escaped from
   * the packed view (pk_vc[0][p] == AM_PK_ESC) with pk_vc[1][p] = i > 0 has its full-width
   * inputs of is_op_in_snapshot/7 in row i - 1 of 2 + n_dc words: commit time, op_meta, then
   * snapshot_time entries by DC -- one contiguous row instead of n_dc + 2 column lines.  An
   * escaped op with pk_vc[1][p] == 0 (written in place since the rows were built) reads the
   * columns.  Escapes are ops with an entry outside the key's 2^32-us window (a DC whose entry
   * lags, e.g. behind a partition) or an invalid effect. */
  const uint64_t *esc_rows;    /* [n_esc][2 + n_dc] or NULL                           */
  /* Lag view (device stores with the packed view, n_dc <= 16, or NULL): an op's commit vector
   * as its commit time and one 16-bit lag per DC -- the snapshot entries of a transaction trail
   * its commit by milliseconds -- so the inclusion test streams 4 + 2 * n_dc bytes per op instead
   * of 4 * n_dc (20 B at D = 8, not 32):
   *   lag_ct[p]     = commit_time - key_tbase[k]   (u32), or AM_PK_ESC when the op is escaped
   *                   from the packed view or one of its lags does not fit
   *   lag[d][p]     = (commit_time - X[d]) - key_lag[k][d]   in [0, 0xFFFF]   (X[dc] = ct: lag 0)
   *   key_lag[k][d] = the smallest commit_time - X[d] over the key's fitting ops (int32)
   * so X[d] - key_tbase[k] = lag_ct[p] - key_lag[k][d] - lag[d][p].  Maintained by every writer
   * (am_store_apply rewrites a touched key's columns and its key_lag row). */
  const uint32_t *lag_ct;      /* [snap_stride]                                       */
  const uint16_t *lag;         /* [n_dc][snap_stride]                                 */
  const int32_t *key_lag;      /* [n_keys][n_dc]                                      */
} am_op_log;
#define AM_ZONE_OPS 256u
#define AM_GMASK_MAX_GRP 32u
#define AM_REC_KILL (1u << 16)
#define AM_REC_OP(m) ((m) & 0xFFFFu)
#define AM_REC_GRP(m) ((m) >> 17)
#define AM_NGRP_NONE 0xFFFFFFFFu
#define AM_GRP_MAX_REC 2048u
/* Chunked token-group view of a hot MV-register key (more than AM_BIG_MIN_OPS ops): its groups
 * are built with device-wide sorts instead of one workgroup's LDS, key_ngrp[k] = G |
 * AM_NGRP_BIG (G < AM_BIG_MAX_GRP), and its record range is laid out per AM_BIG_CHUNK ops:
 *   rec_g[rec_key_off[k] + c], c = 0..nch   the chunk table: record offset (relative to
 *                                           rec_key_off[k]) of the first record of key op
 *                                           c * AM_BIG_CHUNK; entry nch ends the last chunk
 *                                           (nch = ceil(ops / AM_BIG_CHUNK))
 *   then one record per birth / effective kill, in op order:
 *     op within its chunk (bits 0-9) | kill << 10 | group << 11, or 0xFFFFFFFF
 * Groups and their pairs (grp) are as above; an effective kill always follows its group's
 * birth, so a group survives a read iff its birth is included and no kill of it is. */
#define AM_NGRP_BIG 0x80000000u
#define AM_BIG_MIN_OPS (AM_GRP_MAX_REC / 2)
#define AM_BIG_CHUNK 1024u
#define AM_BIG_MAX_GRP (1u << 21)
#define AM_BREC_OP(m) ((m) & 0x3FFu)
#define AM_BREC_KILL (1u << 10)
#define AM_BREC_GRP(m) ((m) >> 11)
#define AM_PK_ESC 0xFFFFFFFFu

/*
 * CRDT values (base snapshots in, materialized values out), SoA over reads.
 *   PN        v0
 *   LWW       v0 = ts (as u64 bits), v1 = value, vflag = 1 for the initial
 *             {0, <<>>} value (a binary sorts above every integer)
 *   AWSET     CSR of (elem, token) pairs: the orddict [{Elem, Tokens}] flattened in
 *             the reference's order (elems ascending, each token list in list order,
 *             the newest add first)
 *   MVREG     CSR of (value, token) pairs sorted (insert_sorted).  set_off[n+1] gives
 *             each read's capacity, set_len[n] the used length.
 *   BCOUNTER  the same CSR, one (slot, value) pair per orddict entry (present iff it was
 *             ever updated): the P orddict {From,To} -> N at slot From*n_dc+To, then the D
 *             orddict Id -> N at slot n_dc*n_dc+Id, each in key order (set_a = slot,
 *             set_b = the int64 value) -- only the touched entries, as the reference's
 *             orddicts hold them (src/bcounter_mgr.erl:80-97 effects), at most
 *             n_dc*n_dc + n_dc per read
 */
typedef struct am_values {
  int64_t *v0;
  uint64_t *v1;
  uint8_t *vflag;
  const uint64_t *set_off;
  uint32_t *set_len;
  uint64_t *set_a;
  uint64_t *set_b;
} am_values;

/* One batch of snapshot reads: the materialize/4 inputs per key. */
typedef struct am_read_batch {
  uint64_t n_reads;
  uint32_t per_read_clock; /* 0: one MinSnapshotTime for the whole batch; 1: one per read */
  uint32_t type_hint;      /* am_type when every read has that type (fast path); 0 = mixed */
  const uint64_t *key;        /* [n] key index into the log                          */
  const uint8_t *type;        /* [n] requested Type                                  */
  const uint64_t *read_vc;    /* [n_dc] or [n_dc][n] MinSnapshotTime                 */
  const uint32_t *read_pres;  /* [1] or [n]                                          */
  const uint64_t *txid;       /* [n] TxId, or NULL => every read's TxId is ignore    */
  const uint8_t *txid_valid;  /* [n] or NULL (all valid when txid != NULL)           */
  /* base snapshot: #snapshot_get_response{snapshot_time, materialized_snapshot} */
  const uint8_t *base_ignore; /* [n] 1 => snapshot_time = ignore; NULL => all ignore  */
  const uint64_t *base_vc;    /* [n_dc][n]                                            */
  const uint32_t *base_pres;  /* [n]                                                  */
  const int64_t *base_last_op;/* [n] or NULL => 0                                     */
  am_values base;             /* NULL members => the type's new() value               */
} am_read_batch;

/* materialize/4 outputs: {ok, Value, NewLastOp, LastOpCt, IsNewSS, Count} */
typedef struct am_read_result {
  int32_t *status;         /* [n] am_status                                */
  int64_t *new_last_op;    /* [n] NewLastOp                                */
  uint64_t *last_ct;       /* [n_dc][n] LastOpCt                           */
  uint32_t *last_ct_pres;  /* [n]                                          */
  uint8_t *last_ct_ignore; /* [n] 1 => LastOpCt = ignore                   */
  uint8_t *is_new_ss;      /* [n]                                          */
  uint32_t *count;         /* [n] number of effects applied                */
  uint8_t *flags;          /* [n] AM_FLAG_*                                */
  am_values value;
} am_read_result;

typedef struct am_ctx am_ctx;     /* device + HIP stream + scratch             */
typedef struct am_store am_store; /* a device-resident op log (one partition)  */
typedef struct am_comm am_comm;   /* RCCL communicator for the GST all-reduce  */

/* ---- context ---- */
int am_abi_version(void);
int am_ctx_open(int device, am_ctx **out);
int am_ctx_close(am_ctx *ctx);
void *am_ctx_stream(am_ctx *ctx);           /* hipStream_t */
int am_ctx_sync(am_ctx *ctx);
const char *am_last_error(void);            /* thread-local message of the last failure */
int am_timer_start(am_ctx *ctx);             /* hipEventRecord on the ctx stream         */
int am_timer_stop(am_ctx *ctx, float *ms);   /* records, syncs, returns elapsed ms       */
/* Counters of the context's kernels (synchronizes the stream): AM_STAT_OPS_SKIPPED = ops whose
 * commit vectors a read did not stream because their zone is inside its base snapshot
 * (am_op_log.zone_vc).  reset != 0 zeroes the counter after reading it. */
#define AM_STAT_OPS_SKIPPED 0
/* token-group records a read did not stream because their zones' group summaries stood in
 * for them (am_op_log.zone_gsum), and the summary words it read instead */
#define AM_STAT_RECS_SKIPPED 1
#define AM_STAT_GSUM_WORDS 2
int am_ctx_stat(am_ctx *ctx, int which, uint64_t *value, int reset);

/* ---- device memory helpers (the NIF owns no framework allocator) ---- */
int am_dev_alloc(am_ctx *ctx, size_t bytes, void **out);
int am_dev_free(am_ctx *ctx, void *p);
int am_memcpy_h2d(am_ctx *ctx, void *dst, const void *src, size_t bytes);
int am_memcpy_d2h(am_ctx *ctx, void *dst, const void *src, size_t bytes);

/* ---- ops cache in HBM ---- */
/* Upload a host op log into device memory owned by the store. */
int am_store_create(am_ctx *ctx, const am_op_log *host_log, am_store **out);
/* Device view of the store (pointers are device pointers). */
int am_store_log(const am_store *st, am_op_log *out);
int am_store_destroy(am_store *st);
/* The zone index of a device store (am_op_log.zone_vc / zone_gsum): level AM_INDEX_NONE drops it,
 * AM_INDEX_ZONES keeps the per-block upper bounds only (base-snapshot reads skip the blocks
 * inside their base; no exact marks), AM_INDEX_EXACT adds the exact marks (fresh reads take an
 * exact block inside their clock whole), AM_INDEX_SUMMARIES adds the group summaries (the
 * default every store builder leaves).  Rebuilds from the op columns; blocks until done.
 * It frees and replaces the store's zone_vc / zone_gsum buffers: an am_op_log obtained from
 * am_store_log before the call holds stale pointers and must be fetched again. */
#define AM_INDEX_NONE 0
#define AM_INDEX_ZONES 1
#define AM_INDEX_EXACT 2
#define AM_INDEX_SUMMARIES 3
int am_store_index(am_ctx *ctx, am_store *st, int level);

/* ---- the hot path ---- */
/* Device pointers; runs on the ctx stream.  Asynchronous except for two data-dependent
 * counter readbacks: a mixed-type batch reads the lane tier's hand-off count once (and
 * returns there when every read was short), and a batch whose set / bounded-counter reads
 * reach the big-read tier reads that tier's count once to size its scratch. */
int am_materialize(am_ctx *ctx, const am_op_log *dev_log, const am_read_batch *dev_batch,
                   am_read_result *dev_res);
/* Host pointers for batch/result; the log is the store's device log.  Blocks. */
int am_materialize_host(am_ctx *ctx, const am_store *st, const am_read_batch *host_batch,
                        am_read_result *host_res);

/* ---- snapshot cache (materializer_vnode snapshot_cache-P) ----
 * Replaces get_from_snapshot_cache/5 + materialize_snapshot/7 + internal_store_ss/4 +
 * snapshot_insert_gc/4 around materialize/4, i.e. materializer_vnode:internal_read/7
 * (src/materializer_vnode.erl:371-376, 384-413, 469-509, 342-364, 515-563) and vector_orddict
 * get_smaller / insert_bigger (src/vector_orddict.erl:75-87, 127-140): per key at most
 * AM_SNAPSHOT_THRESHOLD snapshots, newest first, in HBM.  Every type's value: PN / LWW in
 * the entry, set pairs and bounded-counter slots in a device value pool. */
#define AM_SNAPSHOT_THRESHOLD 10   /* src/materializer_vnode.erl:37 */
#define AM_SNAPSHOT_MIN 3          /* :39 */
#define AM_MIN_OP_STORE_SS 5       /* :47 */
#define AM_SNAPCACHE_ABSENT 0xFFFFFFFFu
typedef struct am_snapcache am_snapcache;
int am_snapcache_create(am_ctx *ctx, uint32_t n_dc, uint64_t n_keys, am_snapcache **out);
int am_snapcache_destroy(am_snapcache *cache);
/* internal_read/7 (ShouldGC = false) for a batch of reads: each read's base comes from the
 * cache (the batch's base members are ignored), materialize/4 runs on it, and the result is
 * written back under materialize_snapshot/7's policy.  Per read status: AM_ERR_COLD_PATH
 * when no cached snapshot is vectorclock:le the read clock; AM_ERR_INVALID for a key read
 * a second time in the same batch (the first read, by index, owns the key; am_vnode_read
 * serves repeated keys in batch order).  The log's n_keys must equal the cache's.  Device
 * pointers; synchronizes once to size the value pool when the batch holds set or
 * bounded-counter reads. */
int am_snapcache_read(am_ctx *ctx, am_snapcache *cache, const am_op_log *dev_log, const am_read_batch *dev_batch,
                      am_read_result *dev_res);
/* The same with internal_read's ShouldGC per read (should_gc [n] or NULL = all false).  When
 * snapshot_insert_gc/4 runs for a key (its dict reached AM_SNAPSHOT_THRESHOLD, or ShouldGC),
 * the dict keeps its newest AM_SNAPSHOT_MIN entries and, if gc_mask is given, gc_mask[key] =
 * 1 with the prune threshold (vectorclock:min over the kept entries) in thr_vc[n_dc][n_keys]
 * / thr_pres[n_keys]: exactly the prune arguments of am_store_update (gc_mask is cleared
 * first). */
int am_snapcache_read_gc(am_ctx *ctx, am_snapcache *cache, const am_op_log *dev_log, const am_read_batch *dev_batch,
                         const uint8_t *should_gc, am_read_result *dev_res, uint8_t *gc_mask, uint64_t *thr_vc,
                         uint32_t *thr_pres);
/* The same with host batch/result (blocks). */
int am_snapcache_read_host(am_ctx *ctx, am_snapcache *cache, const am_store *st, const am_read_batch *host_batch,
                           am_read_result *host_res);
/* One key's entries (newest first) to host arrays of AM_SNAPSHOT_THRESHOLD (vc: x n_dc);
 * *n_entries = AM_SNAPCACHE_ABSENT before the key's first read.  NULL arrays are skipped. */
int am_snapcache_get(am_ctx *ctx, const am_snapcache *cache, uint64_t key, uint32_t *n_entries, uint64_t *vc,
                     uint32_t *pres, int64_t *last_op, int64_t *v0, uint64_t *v1, uint8_t *vflag);
/* Entry e's pool words (set pairs a/b; bounded-counter slot values a + presence pres, P slots
 * From*n_dc+To then D slots): *n_words, at most cap_words copied to the host arrays. */
int am_snapcache_get_value(am_ctx *ctx, const am_snapcache *cache, uint64_t key, uint32_t e, uint32_t cap_words,
                           uint32_t *n_words, uint64_t *a, uint64_t *b, uint8_t *pres);

/* A forced snapshot_insert_gc/4 on every cached key (src/materializer_vnode.erl:519-536): the
 * dict keeps its newest min(n, SNAPSHOT_MIN) entries and Thr = the reference's fold over them
 * (:523-527): Acc = the oldest kept clock, then Acc = vectorclock:min([CT1, Acc]) for each entry
 * newest first, where min([V1, V2]) lowers each DC of V1 to min(V1[dc], V2[dc]) with a DC
 * missing from V2 read as 0 (so while the initial {} snapshot is kept nothing is pruned; evidence
 * in oracle/ref_materializer.py vc_min2).  Device outputs: mask[n_keys] (1 = the key has
 * a threshold), thr_vc[n_dc][n_keys], thr_pres[n_keys] -- exactly the prune arguments of
 * am_store_update (so ops are only pruned below snapshots that stay cached).  n_keys is the
 * cache's: hand the outputs only to am_store_update of a store with the same key count (the
 * thr_vc stride; am_snapcache_read already requires it, Store.update checks it). */
int am_snapcache_gc_threshold(am_ctx *ctx, am_snapcache *cache, uint8_t *mask, uint64_t *thr_vc,
                              uint32_t *thr_pres);

/* ---- one partition's materializer_vnode state: ops cache + snapshot cache ----
 * am_vnode_insert_host runs op_insert_gc/3 (src/materializer_vnode.erl:622-647) for every op
 * of host_ops (a host log over the vnode's keys, each key's ops oldest -> newest; a log over
 * more keys grows the vnode's key space first -- the new keys' tuples appear with their first
 * op, :624-629 -- reads of keys past the key space are AM_ERR_INVALID):
 * NewId = OpCounter + 1, and when Length >= ListLen or NewId rem 50 == 0 the GC read
 * internal_read(Key, Type, Op.snapshot_time, ignore, [], true) runs first (store the
 * snapshot, snapshot_insert_gc/4: keep SNAPSHOT_MIN snapshots, prune_ops below their min,
 * resize ListLen); load_ops/2 (:312-319) replays the log through this call.
 * am_vnode_read_host runs internal_read/7 (:371-376) for a host batch (should_gc [n] or
 * NULL), repeated keys served in batch order.  Reads whose dict reaches SNAPSHOT_THRESHOLD
 * GC the same way.  Both block.  The ops cache keeps room for appends per key: a batch touching
 * a few keys is applied in place at O(those keys' ops) (am_store_apply); a key that outgrows its
 * room rebuilds the store once, regrowing every key's room (am_vnode_stats counts both). */
typedef struct am_vnode am_vnode;
int am_vnode_create(am_ctx *ctx, uint32_t n_dc, uint64_t n_keys, am_vnode **out);
int am_vnode_destroy(am_vnode *v);
int am_vnode_insert_host(am_vnode *v, const am_op_log *host_ops);
int am_vnode_read_host(am_vnode *v, const am_read_batch *host_batch, const uint8_t *should_gc,
                       am_read_result *host_res);
/* the vnode's current store and snapshot cache (borrowed; the store changes on GC) */
int am_vnode_parts(am_vnode *v, am_store **st, am_snapcache **sc);
/* ingestion counters: whole-store rebuilds (a key outgrew its room for appends, or the first
 * insert) and in-place applies of the touched keys (am_store_apply, the common case) */
int am_vnode_stats(am_vnode *v, uint64_t *rebuilds, uint64_t *in_place);
/* the ops-cache tuple header of a key: {Length, ListLen} and OpCounter (element 3) */
int am_vnode_key_info(am_vnode *v, uint64_t key, uint64_t *length, uint64_t *list_len, uint64_t *op_counter);

/* ---- read_objects: one transaction's reads over a node's partitions, one call ----
 * clocksi_interactive_coord's read_objects fan-out (src/clocksi_interactive_coord.erl:
 * 732-747) sends one read per key to its partition's read server, which calls
 * materializer_vnode:read/6 (src/clocksi_readitem_server.erl:217-228).  Here the partitions
 * a GPU owns share one vnode whose key space concatenates theirs: partition p owns vnode
 * keys [part_key_base[p], part_key_base[p+1]).  Request i reads partition part[i]'s local
 * key host_batch->key[i]; every request of every partition is ONE internal_read/7 batch
 * (snapshot cache, materialize/4, write-back), results in request order (repeated keys in
 * request order).  A request outside its partition's range gets AM_ERR_INVALID.
 * am_read_objects_submit returns at once; the read runs on a worker thread and
 * am_ticket_wait returns its status (and frees the ticket).  Every buffer the batch and the
 * result point to must stay valid until then. */
typedef struct am_ticket am_ticket;
int am_read_objects_host(am_vnode *v, uint32_t n_parts, const uint64_t *part_key_base, const uint32_t *part,
                         const am_read_batch *host_batch, am_read_result *host_res);
int am_read_objects_submit(am_vnode *v, uint32_t n_parts, const uint64_t *part_key_base, const uint32_t *part,
                           const am_read_batch *host_batch, am_read_result *host_res, am_ticket **out);
int am_ticket_wait(am_ticket *t);

/* ---- op-cache ingestion + garbage collection ----
 * Builds a new store from `st` (st is unchanged; destroy it when no read uses it):
 *   1. prune_ops/2 (src/materializer_vnode.erl:565-604): for keys with prune_mask[k] != 0
 *      only ops with materializer:belongs_to_snapshot_op(Thr_k, CommitTime, SnapshotTime)
 *      (src/materializer.erl:102-106) survive, in order, keeping their op ids;
 *   2. op_insert_gc/3 (:622-647): the ops of dev_new (CSR over the same keys, oldest ->
 *      newest; its op_id column is ignored) are appended with ids OpCounter+1, +2, ...
 * Either step may be skipped (dev_new / prune_mask NULL).  Device pointers: prune_mask
 * [n_keys], thr_vc [n_dc][n_keys], thr_pres [n_keys]; gc_flags [n_keys] (or NULL) receives
 * AM_GC_* per key.  Differences from the ETS tuple: no ListLen sizing (the log is exactly
 * sized), and a key whose ops are all pruned keeps 0 ops (flag AM_GC_PRUNED_ALL) where
 * prune_ops keeps element(FIRST_OP+Len), a 0 placeholder (:580-583).  Blocks. */
#define AM_GC_PRUNED_ALL 0x1u  /* check_filter kept nothing (NewSize == 0, :580), empty logs too */
#define AM_GC_TRIGGER 0x2u     /* some NewId rem OPS_THRESHOLD == 0: op_insert_gc would have
                                  run a GC read (:635) -- the caller's cue to prune next    */
#define AM_OPS_THRESHOLD 50    /* src/materializer_vnode.erl:41 */
int am_store_update(am_ctx *ctx, const am_store *st, const am_op_log *dev_new, const uint8_t *prune_mask,
                    const uint64_t *thr_vc, const uint32_t *thr_pres, uint8_t *gc_flags, am_store **out);

/* In-place ingestion + GC (the vnode's path; src/materializer_vnode.erl:515-647 per touched key).
 * am_store_reserve: a copy of st whose keys have room for appends (key_end / rec_key_end set: a
 * quarter of each key's ops and at least 4 free op slots, variable words and records in
 * proportion), the ETS tuple's ListLen slack (:540-560).  Blocks.
 * am_store_apply: on a store with room, the same prune + append as am_store_update, for the
 * n_touched keys keys[] (device, distinct) only, written into their room in place: dev_new is
 * CSR over the n_touched keys (entry i = keys[i]; or NULL), prune_mask / thr_vc / thr_pres are
 * over the store's n_keys as in am_store_update (or NULL), gc_flags [n_touched] (device, or
 * NULL) receives AM_GC_*.  Cost O(the touched keys' ops).  *applied = 0 when some touched key
 * would outgrow its room (or the store has none): nothing is written, and the caller rebuilds
 * with am_store_update (+ am_store_reserve).  Readers of the store must not run concurrently
 * (the context lock serializes library calls).  Blocks.  A call that fails (AM_ERR_INVALID: a
 * touched key outside the store or repeated) writes nothing into the store; gc_flags is then
 * unspecified. */
int am_store_reserve(am_ctx *ctx, const am_store *st, am_store **out);
int am_store_apply(am_ctx *ctx, am_store *st, uint64_t n_touched, const uint64_t *keys, const am_op_log *dev_new,
                   const uint8_t *prune_mask, const uint64_t *thr_vc, const uint32_t *thr_pres, uint8_t *gc_flags,
                   int *applied);

/* ---- GST (global stable time) ---- */
/* lanes[0..n_dc-1] = per-DC min over the partitions that have the DC (absent = UINT64_MAX);
 * if any partition is undefined every present lane is 0 (get_min_time's rule);
 * lanes[n_dc] = 1 (defined).  Device pointers: part_vc [n_part][n_dc] (partition-major),
 * part_pres [n_part], part_undef [n_part] (or NULL). */
int am_gst_local_min(am_ctx *ctx, uint32_t n_dc, uint32_t n_part, const uint64_t *part_vc,
                     const uint32_t *part_pres, const uint8_t *part_undef, uint64_t *lanes);
/* RCCL communicator (one process per GPU). */
int am_comm_unique_id(void *id_out /* 128 bytes */);
int am_comm_init(am_ctx *ctx, int rank, int nranks, const void *id /* 128 bytes */, am_comm **out);
int am_comm_destroy(am_comm *comm);
/* In place element-wise min of n_dc+1 u64 lanes across ranks (ncclMin/ncclUint64). */
int am_gst_allreduce(am_comm *comm, uint64_t *lanes, uint32_t n_dc);
/* Turn merged lanes into the stable snapshot: undefined => present lanes 0; then the
 * monotone update against last (last_vc/last_pres device, updated in place);
 * gr != 0 additionally replicates the min over present DCs to every present DC
 * (the value a reader gets from get_stable_snapshot/0).  out_vc/out_pres receive the
 * snapshot a reader would use; changed (device u8) = update_stable's Bool. */
int am_gst_finalize(am_ctx *ctx, uint32_t n_dc, const uint64_t *lanes, uint64_t *last_vc,
                    uint32_t *last_pres, int gr, uint64_t *out_vc, uint32_t *out_pres,
                    uint8_t *changed);

/* CPU twins of am_gst_local_min / the all-reduce's element-wise min / am_gst_finalize, compiled
 * from the same per-DC code as the kernels (am_gst.hip): host pointers, no device.  A node
 * whose GST merge runs on the host (and the multi-process tests, which exchange lanes over
 * gloo) gets the device path's exact encoding and rules. */
int am_gst_local_min_host(uint32_t n_dc, uint32_t n_part, const uint64_t *part_vc, const uint32_t *part_pres,
                          const uint8_t *part_undef, uint64_t *lanes);
int am_gst_merge_lanes_host(uint32_t n_dc, const uint64_t *in, uint64_t *inout);  /* inout = min(in, inout), n_dc+1 lanes */
int am_gst_finalize_host(uint32_t n_dc, const uint64_t *lanes, uint64_t *last_vc, uint32_t *last_pres, int gr,
                         uint64_t *out_vc, uint32_t *out_pres, uint8_t *changed);

/* ---- sharding ---- */
/* 0-based partition position for integer keys: abs(K) rem n_partitions. */
uint32_t am_key_partition(int64_t key, uint32_t n_partitions);
/* The same for keys passed as bytes (log_utilities:convert_key/1, src/log_utilities.erl:
 * 100-118): AM_KEY_BINARY -- the key is a binary; its text, if list_to_integer accepts it
 * ([+-]?[0-9]+, any length), gives abs(Int) rem n, else the SHA-1 chash_key path;
 * AM_KEY_TERM -- bytes = term_to_binary(Key) of a key that is neither an integer nor a
 * binary (chash_key({?BUCKET, term_to_binary(Key)})).  chash_key(B) = SHA-1 of
 * term_to_binary({<<"antidote">>, B}); crypto:bytes_to_integer of it rem n. */
#define AM_KEY_BINARY 0
#define AM_KEY_TERM 1
uint32_t am_key_partition_bytes(const uint8_t *bytes, uint64_t len, int kind, uint32_t n_partitions);
/* riak_core_util:chash_key({<<"antidote">>, B}) for a binary B: 20-byte SHA-1 digest */
int am_chash_key(const uint8_t *bytes, uint64_t len, uint8_t out[20]);

/* ---- term codec (am_codec.hip) ----
 * Order-preserving interning of Erlang terms (external term format, enif_term_to_binary)
 * into the u64 LABELS the device holds for LWW values, MV values and tokens, and add-wins-set
 * elements and tokens: label order == Erlang term order, so the device's sorted outputs are
 * the reference's orddict order, and am_codec_term turns labels back into terms.  One codec
 * per partition (or node); thread-safe.  Labels lie in [1, 2^64-2].  Supported terms:
 * integers, floats, atoms, tuples, lists (proper and improper), binaries and bitstrings;
 * maps, pids, ports, references and funs give AM_ERR_UNSUPPORTED.  Terms that compare equal
 * (1 and 1.0) share one label.
 * When a call needs room that the label space no longer has between two neighbours, every
 * label is re-spread (order kept) and *relabeled is set: take the old -> new map with
 * am_codec_take_relabel and apply it with am_store_relabel / am_snapcache_relabel /
 * am_vnode_relabel to every structure holding labels BEFORE putting this call's labels on
 * the device.  Until the map is taken, am_codec_intern fails with AM_ERR_INVALID. */
typedef struct am_codec am_codec;
#define AM_CODEC_ABSENT 1 /* am_codec_lookup: the term was never interned */
int am_codec_create(am_codec **out);
int am_codec_destroy(am_codec *c);
int am_codec_intern(am_codec *c, uint64_t n, const uint8_t *const *terms, const uint64_t *lens, uint64_t *labels,
                    int *relabeled);
int am_codec_lookup(am_codec *c, const uint8_t *term, uint64_t len, uint64_t *label);
/* the term of a label (external term format); *len always set; AM_ERR_CAPACITY if cap < len */
int am_codec_term(am_codec *c, uint64_t label, uint8_t *buf, uint64_t cap, uint64_t *len);
uint64_t am_codec_size(am_codec *c);
/* pending relabel map, old labels increasing; old/new NULL: *n = its size only */
int am_codec_take_relabel(am_codec *c, uint64_t *old_labels, uint64_t *new_labels, uint64_t cap, uint64_t *n);
/* Erlang term order of two encoded terms: *out = -1, 0, 1 */
int am_codec_compare(const uint8_t *a, uint64_t la, const uint8_t *b, uint64_t lb, int *out);
/* apply a relabel map (host arrays from am_codec_take_relabel) in place: the store's LWW
 * values, MV values and tokens, AW elements and tokens, and its token-group view */
int am_store_relabel(am_ctx *ctx, am_store *st, const uint64_t *old_labels, const uint64_t *new_labels, uint64_t n);
/* the same for a snapshot cache: LWW values and the set pairs in the value pool; key_type is
 * the device key-type column of the store the cache serves ([n_keys]) */
int am_snapcache_relabel(am_ctx *ctx, am_snapcache *c, const uint8_t *key_type, const uint64_t *old_labels,
                         const uint64_t *new_labels, uint64_t n);
/* both, for a vnode's ops cache and snapshot cache */
int am_vnode_relabel(am_vnode *v, const uint64_t *old_labels, const uint64_t *new_labels, uint64_t n);

/* ---- transaction ids (am_txid.hip) ----
 * is_op_in_snapshot/7 compares TxIds for equality only: TxId == Op#clocksi_payload.txid
 * (src/clocksi_materializer.erl:232).  #tx_id{local_start_time, server_pid}
 * (include/antidote.hrl:192-195) holds a pid, so TxIds are NOT labelled by the ordered codec:
 * am_txid_intern maps the external term format of a TxId (enif_term_to_binary, pids, ports and
 * references included) to a dense u64 id, the op_txid / am_read_batch.txid words.  Every
 * encoding of one term gets one id (the bytes are canonicalised first); ids start at 1, are
 * never reordered, relabeled or reused.  am_txid_forget drops an ended transaction's entry.
 * Thread-safe.  Maps and funs: AM_ERR_UNSUPPORTED.
 * Lifetime: a reader's TxId (am_txid_intern) is HELD until am_txid_forget; an op's TxId
 * (am_txid_intern_op, stamped with the op's commit_time {DcId, CT}, DcId as a DC index) is
 * dropped by am_txid_expire once the stable snapshot covers CT and no reader holds it -- the
 * transaction has committed everywhere, so no live read carries it (ops replicated from other
 * DCs, whose TxIds no local coordinator forgets, leave the map this way).  Replaces the
 * #clocksi_payload.txid bookkeeping of materializer_vnode:update/2 (src/materializer_vnode.erl:106-110)
 * and the TxId test of is_op_in_snapshot/7 (src/clocksi_materializer.erl:232). */
typedef struct am_txids am_txids;
int am_txid_create(am_txids **out);
int am_txid_destroy(am_txids *t);
int am_txid_intern(am_txids *t, const uint8_t *term, uint64_t len, uint64_t *id);
int am_txid_intern_op(am_txids *t, const uint8_t *term, uint64_t len, uint32_t dc, uint64_t ct, uint64_t *id);
/* AM_CODEC_ABSENT when the TxId was never interned (or was forgotten / expired) */
int am_txid_lookup(am_txids *t, const uint8_t *term, uint64_t len, uint64_t *id);
int am_txid_forget(am_txids *t, const uint8_t *term, uint64_t len);
/* drop the unheld op entries whose commit time the stable snapshot (stable_vc[n_dc], presence
 * bits stable_pres: the GST, stable_time_functions:get_min_time/1) covers; *dropped (or NULL) */
int am_txid_expire(am_txids *t, uint32_t n_dc, const uint64_t *stable_vc, uint32_t stable_pres, uint64_t *dropped);
uint64_t am_txid_size(am_txids *t);
/* the canonical encoding the map keys on (131-prefixed); *out_len always set */
int am_txid_canonical(const uint8_t *term, uint64_t len, uint8_t *buf, uint64_t cap, uint64_t *out_len);

/* ---- synthetic op logs (bench + parity; counter-based, regenerable per key) ---- */
typedef struct am_synth_params {
  uint64_t seed;
  uint64_t n_keys;
  uint32_t ops_per_key;  /* uniform log length (ignored when zipf_milli != 0)  */
  uint32_t n_dc;
  uint32_t type;         /* am_type, or 0 for mixed (40/20/20/20 PN/LWW/AW/MV),
                            or 6 for MV register + bounded counter (50/50)    */
  uint32_t key_base;     /* global index of key 0 (for sharding)               */
  uint32_t max_lag;      /* snapshot lag in ops (concurrency window)           */
  uint32_t zipf_milli;   /* Zipf exponent x1000 for key popularity; 0 = uniform */
  uint64_t total_ops;    /* Zipf: target total ops over all keys               */
  uint32_t hot_cap;      /* Zipf: cap on one key's log length                  */
  uint32_t universe;     /* AW-set element universe per key (power of two)     */
  uint64_t part_mask;    /* 0: local key k is global key key_base + k.  Else the
                            riak_core partitions (of 64) this GPU owns: local key
                            k is the k-th integer key >= key_base whose partition
                            am_key_partition(key, 64) = key mod 64 is in the mask */
  uint32_t esc_ppm;      /* ops (per 10^6) whose snapshot_time holds one remote DC's entry
                            2^33 us behind: outside the packed view's window (escaped ops) */
  uint32_t _pad2;
} am_synth_params;
#define AM_SYNTH_MV_BC 6
/* Device log owned by the returned store. */
int am_synth_store(am_ctx *ctx, const am_synth_params *p, am_store **out);
/* The read clock the generator's quantile q selects (q in [0,1]); host output [n_dc]. */
int am_synth_read_clock(const am_synth_params *p, double q, uint64_t *out_vc);
/* The global key of local key k (see part_mask). */
uint64_t am_synth_key(const am_synth_params *p, uint64_t k);
/* Regenerate keys [k0, k0+nk) on the host into caller buffers sized by
 * am_synth_host_sizes (for parity checks against the oracle). */
int am_synth_host_sizes(const am_synth_params *p, uint64_t k0, uint64_t nk, uint64_t *n_ops,
                        uint64_t *n_var);
int am_synth_host(const am_synth_params *p, uint64_t k0, uint64_t nk, am_op_log *out_host_bufs);

#ifdef __cplusplus
}
#endif
#endif /* ANTIDOTE_MAT_H */
