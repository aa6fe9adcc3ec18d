// am_internal.h -- shared internals of libantidote_mat (not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "../../include/antidote_mat.h"

enum { AM_SCR_PLAN = 0, AM_SCR_BIGMETA = 1, AM_SCR_BIGREC = 2, AM_SCR_ROWS = 3, AM_SCR_GRP = 4, AM_SCR_SPARE = 5, AM_SCR_SNAP = 6, AM_SCR_GC = 7, AM_SCR_SIZES = 8, AM_SCR_MISC = 9, AM_SCR_INCL = 10, AM_N_SCR = 11 };

struct am_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  int n_cu = 256;
  void *scratch[AM_N_SCR] = {};  // grow-only device scratch slots (planner, row/group hand-offs, big-read path)
  size_t scratch_bytes[AM_N_SCR] = {};
  uint64_t *pinned = nullptr;    // small pinned host buffer for device -> host counters
  uint64_t *stats = nullptr;     // device counters (am_ctx_stat: AM_STAT_*)
  // Device blocks of destroyed stores / caches kept for reuse by am_dev_alloc (a rebuilt
  // store -- am_store_update every GC round -- asks for the same column sizes again), by
  // size; block sizes of every am_dev_alloc block.  Reuse is stream-ordered: every kernel
  // of the context runs on its one stream.
  std::multimap<size_t, void *> free_blocks;
  std::unordered_map<void *, size_t> block_size;
  size_t free_bytes = 0;
  // Every entry point that touches the stream, the scratch slots or the pinned buffer holds
  // this lock, so concurrent callers on one context (a partition's READ_CONCURRENCY read
  // servers, include/antidote.hrl:28) serialize instead of sharing scratch; recursive
  // because composite calls (am_vnode_*, the *_host wrappers) re-enter.
  std::recursive_mutex mu;
  // A snapshot-cache read (am_snapcache.hip sets these around its am_launch_materialize
  // call, null otherwise):
  //   grp_hint_in[w]  the token group of cached base word w in the log it was cached from
  //                   (used only after its pair matches the group's pair in the current log,
  //                   so a stale hint costs a search, never a wrong answer)
  //   tee_*           the wave kernel also writes every value word it outputs (result word o)
  //                   into the cache's pool at word o + tee_shift, with its group, and sets
  //                   tee_done[r]; k_sc_store then links a stored snapshot to those words
  //                   instead of copying them
  const uint32_t *grp_hint_in = nullptr;
  uint64_t *tee_a = nullptr, *tee_b = nullptr;
  uint32_t *tee_g = nullptr;
  int64_t tee_shift = 0;
  uint8_t *tee_done = nullptr;
  // The mixed-batch planner's per-type streams (am_plan.hip): sub-contexts of the set types
  // (and [3]: the big-MV reads started beside the lane tier) on the same device, sharing the
  // counters, each with its own stream, scratch slots and pinned buffer, so one type's tiers
  // overlap another's.  ev_fork orders them after the
  // planner; their ev0 joins them back.
  am_ctx *sub[4] = {};
  bool is_sub = false;
  hipEvent_t ev_fork = nullptr;
  // the CRDT types present in a log's keys, by key_type array: {n_keys, 1 << type mask}
  std::unordered_map<const void *, std::pair<uint64_t, uint32_t>> type_masks;
};
// sub-context i of c (created on first use; null on failure, error set)
am_ctx *am_ctx_sub(am_ctx *c, int i);
#define AM_LOCK(ctxp) std::lock_guard<std::recursive_mutex> am_lock_((ctxp)->mu)

// A selection of a batch's reads: the planner's per-kernel sub-batches.  idx == nullptr
// means the identity over [0, n_reads); otherwise the reads idx[range[0] .. range[1])
// (range lives in device memory, so sub-batch sizes never round-trip to the host).
struct am_sel {
  const uint32_t *idx = nullptr;
  const uint32_t *range = nullptr;
};
// Reads a set kernel could not finish in LDS (appended by the kernel; count on device).
struct am_retry {
  uint32_t *list = nullptr;
  uint32_t *count = nullptr;
};

// scratch slot `slot` (0 planner, 1 big-read metadata, 2 big-read records): at least
// `bytes` of device memory, valid until the next call for the same slot (stream-ordered
// reuse; growing synchronizes the stream before freeing the old block)
int am_ctx_scratch(am_ctx *ctx, int slot, size_t bytes, void **out);
// copy `n` u64 counters device -> host through the pinned buffer (synchronizes the stream)
int am_ctx_fetch(am_ctx *ctx, const void *dev, uint32_t n_u64, uint64_t *host);

// return an am_dev_alloc block to the context (kept for reuse, or freed past the cache cap)
extern "C" void am_dev_release(am_ctx *ctx, void *p);

struct am_store {
  am_ctx *ctx = nullptr;
  am_op_log dev{};               // device view
  std::vector<void *> allocs;    // owned device allocations
  uint64_t *counter = nullptr;   // [n_keys] OpCounter (ops-cache tuple element 3) after
                                 // am_store_update; null => the newest op's id
  int zone_level = AM_INDEX_SUMMARIES;  // the zone index it keeps (am_store_index)
};
// zone_vc rows after the n_dc maxima: exact mark, summary offset, records end, records begin,
// summary slot (include/antidote_mat.h)
constexpr uint32_t AM_ZONE_EXTRA_ROWS = 5;
// bounded-counter reads of longer logs go to the chunked big-read tier (am_bcwave.hip: a wave
// streaming 32768 ops alone was the tail of C5 at a 32768 limit)
constexpr uint64_t AM_BCWAVE_OPS = 4096;
// the LDS-sort tier (am_sets.hip) hands logs longer than this to the big-read tier whole
constexpr uint64_t AM_SETS_BIG_OPS = 4096;

void am_set_error(const char *fmt, ...);

// the end of key k's ops / records (include/antidote_mat.h: key_end / rec_key_end, the room
// for appends of a vnode store; without them the CSR's next offset)
__host__ __device__ __forceinline__ uint64_t am_kend(const am_op_log &L, uint64_t k) {
  return L.key_end ? L.key_end[k] : L.key_off[k + 1];
}
__host__ __device__ __forceinline__ uint64_t am_rkend(const am_op_log &L, uint64_t k) {
  return L.rec_key_end ? L.rec_key_end[k] : L.rec_key_off[k + 1];
}

#define AM_HIP(call)                                                                  \
  do {                                                                                \
    hipError_t e_ = (call);                                                           \
    if (e_ != hipSuccess) {                                                           \
      am_set_error("%s:%d %s -> %s", __FILE__, __LINE__, #call, hipGetErrorString(e_)); \
      return AM_ERR_HIP;                                                              \
    }                                                                                 \
  } while (0)

// ops are padded so every per-op array can be read in groups of 4 (32 B of u64)
static constexpr uint64_t AM_OP_PAD = 256;
static inline uint64_t am_round_up(uint64_t x, uint64_t m) { return (x + m - 1) / m * m; }

// internal launchers (am_materialize.hip, am_gst.hip, am_synth.hip)
int am_launch_materialize(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R);
int am_launch_gst_local_min(am_ctx *ctx, uint32_t n_dc, uint32_t n_part, const uint64_t *part_vc,
                            const uint32_t *part_pres, const uint8_t *part_undef, uint64_t *lanes);
int am_launch_gst_finalize(am_ctx *ctx, uint32_t n_dc, const uint64_t *lanes, uint64_t *last_vc,
                           uint32_t *last_pres, int gr, uint64_t *out_vc, uint32_t *out_pres,
                           uint8_t *changed);
int am_launch_synth(am_ctx *ctx, const am_synth_params *p, am_op_log *L /* device arrays allocated */);
int am_launch_stream(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S,
                     uint32_t type);
int am_launch_sets(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S,
                   uint32_t type, am_retry retry);
int am_launch_big(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, uint32_t type,
                  am_retry retry);  // am_big.hip: reads beyond the LDS tier
// Token-group tier (am_group.hip) for add-wins-set / MV-register reads over the packed view
// and the token-group view, three kernels by read size: AM_GRP_ROW (16-lane row per short
// log), AM_GRP_WAVE (wave per read), AM_GRP_WG (512-thread workgroup per read).  Reads a
// kernel does not take (ungrouped keys, base-snapshot pairs, logs beyond its limits) go to
// `next`.
enum { AM_GRP_ROW = 0, AM_GRP_WAVE = 1, AM_GRP_WG = 2 };
// with AM_GRP_WAVE: hand the reads the lane tier takes (<= 64 ops, <= 64 groups) to `next`
constexpr int AM_GRP_HAND_SHORT = 0x100;
bool am_group_applies(const am_op_log *L, const am_read_result *R, uint32_t type);
int am_launch_group(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S,
                    uint32_t type, am_retry next, int tier);
// Lane tier (am_lanes.hip): one lane per short read of the PN counter, LWW register,
// add-wins set and MV register, every accepted type in one launch.  accept = bit mask
// (1 << am_type) of the types it may take; am_lane_accept() narrows a wish list to the types
// the log and the outputs support (packed view; value columns; token-group view).  Reads
// it does not take go to `next`; unknown keys / types and corrupted logs get their status.
uint32_t am_lane_accept(const am_op_log *L, const am_read_result *R, uint32_t types);
int am_launch_lanes(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S,
                    am_retry next, uint32_t accept);
// Short bounded-counter reads (am_bcrows.hip): one 16-lane row per read of <= 64 ops, batch
// clock, packed view, n_dc <= 16; the touched slots only (bitmap ranks, compact sums).  Longer
// reads (and the few with an |amount| >= 2^56) go to `next`.
bool am_bcrows_applies(const am_op_log *L, const am_read_batch *B, const am_read_result *R);
int am_launch_bcrows(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S,
                     am_retry next);
// Bounded-counter wave tier (am_bcwave.hip): one wave per read with LDS slot sums, reads
// up to 4096 ops over the packed view (n_dc <= 16); the rest go to `next`.
bool am_bcwave_applies(const am_op_log *L, const am_read_result *R);
int am_launch_bcwave(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S,
                     am_retry next);
// the token-group view of a store (per-op record offsets rcnt [n_ops+1], rec_key_off set in L)
int am_launch_group_build(am_ctx *ctx, const am_op_log *L, const uint64_t *rcnt, uint32_t *rec_g, uint64_t *grp,
                          uint32_t *key_ngrp, uint64_t *prec);
// the chunked token-group view of the hot MV keys (am_grpbig.hip), after am_launch_group_build
int am_launch_group_build_big(am_ctx *ctx, const am_op_log *L, const uint64_t *rcnt, uint32_t *rec_g, uint64_t *grp,
                              uint32_t *key_ngrp);
int am_store_pack(am_store *st);  // builds the packed streaming view (am_pack.hip)
// am_store_update over a log view (am_gc.hip): counter = OpCounter per key or null; slack =>
// the new store has room for appends (key_end / rec_key_end set, am_store_apply), at least
// cap_hint[k] op slots for key k when cap_hint (device [n_keys]) is given
int am_store_update_ex(am_ctx *c, const am_op_log &L, const uint64_t *counter, const am_op_log *dev_new,
                       const uint8_t *prune_mask, const uint64_t *thr_vc, const uint32_t *thr_pres, uint8_t *gc_flags,
                       bool slack, const uint64_t *cap_hint, am_store **out);
// in-place ingestion + GC of the m keys d_keys (device list, distinct) of a slack store
// (am_apply.hip): dev_new = new ops as CSR over the m keys (or null); d_mask_full / thr over the
// store's n_keys (or null); d_gc_flags [m] receives AM_GC_*; h_new_len [m] (host, or null) the
// keys' op counts after.  *applied = 0: some key does not fit its room (nothing written) --
// rebuild the whole store instead.
int am_store_apply_ex(am_ctx *c, am_store *st, uint64_t m, const uint64_t *d_keys, const am_op_log *dev_new,
                   const uint8_t *d_mask_full, const uint64_t *d_thr_vc_full, const uint32_t *d_thr_pres_full,
                   uint8_t *d_gc_flags, uint64_t *h_new_len, int *applied, bool check_keys = false);
int am_store_grow_keys(am_ctx *c, const am_store *st, uint64_t n_new, const uint64_t *cap_hint, am_store **out);  // am_apply.hip
struct am_snapcache;
extern "C" int am_snapcache_grow(am_snapcache *c, uint64_t new_n);  // am_snapcache.hip (not exported in the header)
int am_store_key_lens(am_ctx *c, const am_store *st, uint64_t m, const uint64_t *d_keys, const uint8_t *flags_full,
                      uint64_t *h_len, uint8_t *h_flags);

// Short-read tier (am_rows.hip): reads with at most short_max ops (and error reads) are
// materialized by one 16-lane row each.  list/count (set types only): reads the tier
// leaves to the workgroup tier -- longer logs, and reads whose births/kills overflow
// the row's LDS lists -- appended in batch order (count lives on the device).
// mask (PN/LWW): per 64-read batch of the selection, the reads k_stream left to the row
// tier (bit i = read rb + i); k_stream writes it, the row tier skips batches with 0.
struct am_rows_cfg {
  uint32_t short_max = 0;
  uint32_t *list = nullptr;
  uint32_t *count = nullptr;
  uint64_t *mask = nullptr;
};
int am_launch_rows(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S, uint32_t type,
                   const am_rows_cfg &C);
// k_stream with H.mask set: reads with at most H.short_max ops (and error reads) are
// not materialized but marked in H.mask for the row tier
int am_launch_stream_skip(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S,
                          uint32_t type, const am_rows_cfg &H);
// a key's group count (0 for an ungrouped key) and whether its view is the chunked one
__host__ __device__ __forceinline__ uint32_t am_ngrp_count(uint32_t ng) {
  return ng == AM_NGRP_NONE ? 0u : (ng & ~AM_NGRP_BIG);
}
__host__ __device__ __forceinline__ bool am_ngrp_big(uint32_t ng) {
  return ng != AM_NGRP_NONE && (ng & AM_NGRP_BIG) != 0;
}
// a key that gets the chunked token-group view when its log allows (include/antidote_mat.h):
// an MV register with more than AM_BIG_MIN_OPS ops (an assign births one token and kills the
// ones it overrides, so such a key's records outgrow the LDS builder's AM_GRP_MAX_REC), all of
// one type
__host__ __device__ __forceinline__ bool am_big_grp_key(const am_op_log &L, uint64_t k) {
  return L.key_type[k] == AM_MVREG && am_kend(L, k) - L.key_off[k] > AM_BIG_MIN_OPS &&
         !(L.key_flags && (L.key_flags[k] & AM_KEY_MIXED_TYPES));
}
// the chunk table's words
__host__ __device__ __forceinline__ uint64_t am_big_hdr(uint64_t ops) { return (ops + AM_BIG_CHUNK - 1) / AM_BIG_CHUNK + 1; }

// the batch uses partial clocks, op ids, TxIds, cached bases or per-read clocks
inline bool am_batch_general(const am_op_log *L, const am_read_batch *B) {
  return L->snap_pres || L->op_id || (B->txid && L->op_txid) || B->base_ignore || B->per_read_clock || B->base.v0 ||
         B->base.set_off;
}
// the packed streaming view applies (u32 entries relative to the key time base, full clocks)
inline bool am_log_packed(const am_op_log *L) { return L->key_tbase && L->pk_vc && !L->snap_pres; }
// a relabel map (am_codec_take_relabel) copied to the device; old labels strictly increasing.
// The caller hipFrees both after a stream synchronize.
int am_relabel_upload(am_ctx *c, const uint64_t *old_labels, const uint64_t *new_labels, uint64_t n, uint64_t **d_old,
                      uint64_t **d_new);
