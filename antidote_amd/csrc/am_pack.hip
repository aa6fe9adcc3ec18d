// am_pack.hip -- the packed streaming view of a device op log (am_op_log.ct_meta,
// .snap_delta).  The scan kernels are HBM-bound; the ClockSI inclusion test only
// needs each snapshot entry relative to the op's own commit time, which fits in 32
// bits for any realistic clock lag/skew (2^31 us = 35 min).  Ops that do not fit are
// flagged (AM_CT_ESC) and read from the full columns, so results stay bit-exact.
#include "am_internal.h"

namespace {

__global__ void k_pack(am_op_log L, uint64_t *ct_meta, int32_t *snap_delta) {
  const uint64_t stride = L.snap_stride ? L.snap_stride : L.n_ops;
  const uint32_t all = L.n_dc >= 32 ? 0xFFFFFFFFu : ((1u << L.n_dc) - 1u);
  for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < L.n_ops;
       q += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t ct = L.commit_time[q];
    const uint32_t meta = L.op_meta[q];
    const uint32_t pres = L.snap_pres ? L.snap_pres[q] & all : all;
    bool esc = ct >= AM_CT_ESC;
    for (uint32_t d = 0; d < L.n_dc; ++d) {
      int32_t v = 0;
      if ((pres >> d) & 1u) {
        const uint64_t s = L.snap_vc[(uint64_t)d * stride + q];
        if (s <= ct) {
          const uint64_t diff = ct - s;
          if (diff <= 0x7FFFFFFFull) v = (int32_t)diff;
          else esc = true;
        } else {
          const uint64_t diff = s - ct;
          if (diff <= 0x7FFFFFFFull) v = -(int32_t)diff;
          else esc = true;
        }
      }
      snap_delta[(uint64_t)d * stride + q] = v;
    }
    ct_meta[q] = (esc ? AM_CT_ESC : ct) | ((uint64_t)meta << 56);
  }
}

}  // namespace

int am_store_pack(am_store *st) {
  am_ctx *c = st->ctx;
  am_op_log &d = st->dev;
  const uint64_t stride = d.snap_stride ? d.snap_stride : d.n_ops;
  if (stride % 4 || !d.commit_time || !d.op_meta || (d.n_ops && !d.snap_vc)) return AM_OK;  // not packable
  void *ctm = nullptr, *sd = nullptr;
  int rc = am_dev_alloc(c, stride * 8, &ctm);
  if (rc) return rc;
  st->allocs.push_back(ctm);
  rc = am_dev_alloc(c, (size_t)d.n_dc * stride * 4, &sd);
  if (rc) return rc;
  st->allocs.push_back(sd);
  AM_HIP(hipMemsetAsync(ctm, 0, stride * 8, c->stream));
  AM_HIP(hipMemsetAsync(sd, 0, (size_t)d.n_dc * stride * 4, c->stream));
  if (d.n_ops) {
    const uint64_t blocks = (d.n_ops + 255) / 256 < 65536 ? (d.n_ops + 255) / 256 : 65536;
    hipLaunchKernelGGL(k_pack, dim3((unsigned)blocks), dim3(256), 0, c->stream, d, (uint64_t *)ctm, (int32_t *)sd);
    AM_HIP(hipGetLastError());
  }
  AM_HIP(hipStreamSynchronize(c->stream));
  d.ct_meta = (const uint64_t *)ctm;
  d.snap_delta = (const int32_t *)sd;
  return AM_OK;
}
