// am_gst.hip -- global stable time (GST) on the device + RCCL.
//
// Reference: every partition publishes a stable vectorclock; per node,
// meta_data_sender takes stable_time_functions:get_min_time/1 over the local
// partitions (src/stable_time_functions.erl:51-85), casts that dict to every other
// node, takes the min again over the node dicts (src/meta_data_sender.erl:237-245)
// and applies the monotone update_stable/3 (:342-356).
//
// Here one node = one GPU (one process).  The per-node merge is a tiny kernel
// (am_gst_local_min), the broadcast + node-level min is ONE ncclAllReduce(min,
// uint64) over n_dc+1 lanes on RCCL/xGMI, and the monotone update is
// am_gst_finalize.  Lane encoding: DC d absent -> UINT64_MAX (min-neutral, so an
// absent DC never reads as 0 -- get_min_time only mins over dicts that have the
// DC); lane n_dc = 1 for a defined node dict, 0 for 'undefined' (min = "any
// undefined").  Clock values must therefore be < 2^64 - 1.
#include <rccl/rccl.h>

#include <cstring>

#include "am_internal.h"

namespace {

constexpr uint64_t ABSENT = ~0ull;

// The per-DC steps, shared by the kernels and their CPU twins (am_gst_*_host): one source for
// the device path and the host path the multi-process tests drive.
// get_min_time/1 over one node's partitions, DC d (src/stable_time_functions.erl:51-85)
__host__ __device__ inline uint64_t local_min_dc(uint32_t d, uint32_t n_dc, uint32_t n_part, const uint64_t *vc,
                                                 const uint32_t *pres, const uint8_t *undef) {
  bool any_undef = false, present = false;
  uint64_t m = ABSENT;
  for (uint32_t p = 0; p < n_part; ++p) {
    if (undef && undef[p]) {
      any_undef = true;
      continue;
    }
    if ((pres[p] >> d) & 1u) {
      const uint64_t t = vc[(uint64_t)p * n_dc + d];
      m = (present && m <= t) ? m : t;   // PrevTime >= Time -> store Time
      present = true;
    }
  }
  return present ? (any_undef ? 0 : m) : ABSENT;
}

// meta_data_sender:update_stable/3 with update_func_min/2 (src/meta_data_sender.erl:342-356,
// src/stable_time_functions.erl:42-48), then the gr broadcast (src/dc_utilities.erl:259-277)
__host__ __device__ inline void finalize(uint32_t n_dc, const uint64_t *lanes, uint64_t *last_vc, uint32_t *last_pres,
                                         int gr, uint64_t *out_vc, uint32_t *out_pres, uint8_t *changed) {
  const bool undef = lanes[n_dc] == 0;
  uint32_t lp = *last_pres;
  bool ch = false;
  for (uint32_t d = 0; d < n_dc; ++d) {
    if (lanes[d] == ABSENT) continue;
    const uint64_t t = undef ? 0 : lanes[d];
    // update_func_min(Last, Time): Last undefined -> true; else Time >= Last
    if (!((lp >> d) & 1u) || t >= last_vc[d]) {
      last_vc[d] = t;
      lp |= 1u << d;
      ch = true;
    }
  }
  *last_pres = lp;
  if (changed) *changed = ch ? 1 : 0;
  uint64_t gmin = ABSENT;
  for (uint32_t d = 0; d < n_dc; ++d)
    if ((lp >> d) & 1u) gmin = last_vc[d] < gmin ? last_vc[d] : gmin;
  for (uint32_t d = 0; d < n_dc; ++d) out_vc[d] = ((lp >> d) & 1u) ? (gr ? gmin : last_vc[d]) : 0;
  *out_pres = lp;
}

__global__ void k_gst_local_min(uint32_t n_dc, uint32_t n_part, const uint64_t *vc, const uint32_t *pres,
                                const uint8_t *undef, uint64_t *lanes) {
  const uint32_t d = threadIdx.x;
  if (d < n_dc) lanes[d] = local_min_dc(d, n_dc, n_part, vc, pres, undef);
  if (d == 0) lanes[n_dc] = 1;
}

__global__ void k_gst_finalize(uint32_t n_dc, const uint64_t *lanes, uint64_t *last_vc, uint32_t *last_pres, int gr,
                               uint64_t *out_vc, uint32_t *out_pres, uint8_t *changed) {
  if (threadIdx.x == 0) finalize(n_dc, lanes, last_vc, last_pres, gr, out_vc, out_pres, changed);
}

}  // namespace

int am_launch_gst_local_min(am_ctx *c, uint32_t n_dc, uint32_t n_part, const uint64_t *vc, const uint32_t *pres,
                            const uint8_t *undef, uint64_t *lanes) {
  hipLaunchKernelGGL(k_gst_local_min, dim3(1), dim3(64), 0, c->stream, n_dc, n_part, vc, pres, undef, lanes);
  AM_HIP(hipGetLastError());
  return AM_OK;
}

int am_launch_gst_finalize(am_ctx *c, uint32_t n_dc, const uint64_t *lanes, uint64_t *last_vc, uint32_t *last_pres,
                           int gr, uint64_t *out_vc, uint32_t *out_pres, uint8_t *changed) {
  hipLaunchKernelGGL(k_gst_finalize, dim3(1), dim3(64), 0, c->stream, n_dc, lanes, last_vc, last_pres, gr, out_vc,
                     out_pres, changed);
  AM_HIP(hipGetLastError());
  return AM_OK;
}

struct am_comm {
  am_ctx *ctx = nullptr;
  ncclComm_t comm = nullptr;
  int rank = 0, nranks = 1;
};

#define AM_NCCL(call)                                                                      \
  do {                                                                                     \
    ncclResult_t r_ = (call);                                                              \
    if (r_ != ncclSuccess) {                                                               \
      am_set_error("%s:%d %s -> %s", __FILE__, __LINE__, #call, ncclGetErrorString(r_)); \
      return AM_ERR_RCCL;                                                                  \
    }                                                                                      \
  } while (0)

extern "C" {

int am_comm_unique_id(void *id_out) {
  if (!id_out) return AM_ERR_INVALID;
  ncclUniqueId u;
  AM_NCCL(ncclGetUniqueId(&u));
  std::memcpy(id_out, &u, sizeof(u));
  return AM_OK;
}

int am_comm_init(am_ctx *ctx, int rank, int nranks, const void *id, am_comm **out) {
  if (!ctx || !id || !out || nranks < 1 || rank < 0 || rank >= nranks) return AM_ERR_INVALID;
  AM_HIP(hipSetDevice(ctx->device));
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  am_comm *c = new am_comm();
  c->ctx = ctx;
  c->rank = rank;
  c->nranks = nranks;
  ncclResult_t r = ncclCommInitRank(&c->comm, nranks, u, rank);
  if (r != ncclSuccess) {
    am_set_error("ncclCommInitRank: %s", ncclGetErrorString(r));
    delete c;
    return AM_ERR_RCCL;
  }
  *out = c;
  return AM_OK;
}

int am_comm_destroy(am_comm *c) {
  if (!c) return AM_OK;
  if (c->comm) ncclCommDestroy(c->comm);
  delete c;
  return AM_OK;
}

int am_gst_local_min_host(uint32_t n_dc, uint32_t n_part, const uint64_t *part_vc, const uint32_t *part_pres,
                          const uint8_t *part_undef, uint64_t *lanes) {
  if (!lanes || n_dc > AM_MAX_DC || (n_part && (!part_vc || !part_pres))) return AM_ERR_INVALID;
  for (uint32_t d = 0; d < n_dc; ++d) lanes[d] = local_min_dc(d, n_dc, n_part, part_vc, part_pres, part_undef);
  lanes[n_dc] = 1;
  return AM_OK;
}

int am_gst_merge_lanes_host(uint32_t n_dc, const uint64_t *in, uint64_t *inout) {
  if (!in || !inout || n_dc > AM_MAX_DC) return AM_ERR_INVALID;
  for (uint32_t d = 0; d <= n_dc; ++d) inout[d] = in[d] < inout[d] ? in[d] : inout[d];  // ncclMin on ncclUint64
  return AM_OK;
}

int am_gst_finalize_host(uint32_t n_dc, const uint64_t *lanes, uint64_t *last_vc, uint32_t *last_pres, int gr,
                         uint64_t *out_vc, uint32_t *out_pres, uint8_t *changed) {
  if (!lanes || !last_vc || !last_pres || !out_vc || !out_pres || n_dc > AM_MAX_DC) return AM_ERR_INVALID;
  finalize(n_dc, lanes, last_vc, last_pres, gr, out_vc, out_pres, changed);
  return AM_OK;
}

int am_gst_allreduce(am_comm *c, uint64_t *lanes, uint32_t n_dc) {
  if (!c || !lanes || n_dc > AM_MAX_DC) return AM_ERR_INVALID;
  AM_HIP(hipSetDevice(c->ctx->device));
  AM_NCCL(ncclAllReduce(lanes, lanes, (size_t)n_dc + 1, ncclUint64, ncclMin, c->comm, c->ctx->stream));
  return AM_OK;
}

}  // extern "C"
