// am_stream.hip -- launchers of the streaming materialize kernel (am_stream.h) for the
// PN counter and the LWW register.
#include "am_stream.h"

using namespace amk;
using namespace amk_stream;

namespace {

template <int D, int TYPE, bool GENERAL, bool PACKED>
int launch_d(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S, const am_rows_cfg &H) {
  // persistent-style grid: at most the resident capacity, at most one wave per 64-read batch
  static int occ = 0;
  if (occ == 0) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_stream<D, TYPE, GENERAL, PACKED>, BLOCK, 0) != hipSuccess ||
        nb <= 0)
      nb = 2;
    occ = nb;
  }
  const uint64_t batches = (B->n_reads + WAVE - 1) / WAVE;
  uint64_t blocks = (batches + WPB - 1) / WPB;
  const uint64_t cap = (uint64_t)ctx->n_cu * (uint64_t)occ;
  if (blocks > cap) blocks = cap;
  if (blocks == 0) return AM_OK;
  hipLaunchKernelGGL((k_stream<D, TYPE, GENERAL, PACKED>), dim3((unsigned)blocks), dim3(BLOCK), 0, ctx->stream, *L, *B,
                     *R, S, H);
  AM_HIP(hipGetLastError());
  return AM_OK;
}

template <int TYPE, bool GENERAL, bool PACKED>
int launch(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S, const am_rows_cfg &H) {
  const uint32_t nd = L->n_dc;
  if (nd <= 1) return launch_d<1, TYPE, GENERAL, PACKED>(ctx, L, B, R, S, H);
  if (nd <= 2) return launch_d<2, TYPE, GENERAL, PACKED>(ctx, L, B, R, S, H);
  if (nd <= 3) return launch_d<3, TYPE, GENERAL, PACKED>(ctx, L, B, R, S, H);
  if (nd <= 4) return launch_d<4, TYPE, GENERAL, PACKED>(ctx, L, B, R, S, H);
  if (nd <= 8) return launch_d<8, TYPE, GENERAL, PACKED>(ctx, L, B, R, S, H);
  if (nd <= 16) return launch_d<16, TYPE, GENERAL, PACKED>(ctx, L, B, R, S, H);
  return launch_d<32, TYPE, GENERAL, PACKED>(ctx, L, B, R, S, H);
}

}  // namespace

// FAST variant when the batch uses none of: partial snapshot clocks, explicit op
// ids, TxIds, cached bases, per-read clocks (the bench's fresh snapshot read).
// With a selection (planner sub-batch) the read count lives on the device: the grid is
// the resident capacity and surplus waves exit at once.
int am_launch_stream_skip(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S,
                          uint32_t type, const am_rows_cfg &H) {
  const bool general = am_batch_general(L, B);
  // packed view: streaming bytes per op 8 + 4*D + payload instead of 9 + 8*D + payload
  const bool packed = am_log_packed(L);
  switch (type) {
    case AM_PN:
      if (general)
        return packed ? launch<AM_PN, true, true>(ctx, L, B, R, S, H)
                      : launch<AM_PN, true, false>(ctx, L, B, R, S, H);
      return packed ? launch<AM_PN, false, true>(ctx, L, B, R, S, H)
                    : launch<AM_PN, false, false>(ctx, L, B, R, S, H);
    case AM_LWW:
      if (general)
        return packed ? launch<AM_LWW, true, true>(ctx, L, B, R, S, H)
                      : launch<AM_LWW, true, false>(ctx, L, B, R, S, H);
      return packed ? launch<AM_LWW, false, true>(ctx, L, B, R, S, H)
                    : launch<AM_LWW, false, false>(ctx, L, B, R, S, H);
    default:
      return AM_ERR_UNSUPPORTED;
  }
}

int am_launch_stream(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R, am_sel S,
                     uint32_t type) {
  return am_launch_stream_skip(ctx, L, B, R, S, type, am_rows_cfg{});
}

