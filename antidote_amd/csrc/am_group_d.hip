// am_group_d.hip -- the token-group read kernels (am_group.h) for one clock width, built
// once per D (-DGRP_D=1,2,3,4,8,16,32) so the instantiations compile in parallel.
#include "am_group.h"

#ifndef GRP_D
#error "build with -DGRP_D=<clock width>"
#endif
#define AM_CAT2(a, b) a##b
#define AM_CAT(a, b) AM_CAT2(a, b)

int AM_CAT(am_grp_launch_d, GRP_D)(am_ctx *ctx, const am_op_log *L, const am_read_batch *B, am_read_result *R,
                                   am_sel S, uint32_t type, am_retry next, int tier) {
  using namespace amk_grp;
  if (type == AM_AWSET) return launch_v<GRP_D, AM_AWSET>(ctx, L, B, R, S, next, tier);
  if (type == AM_MVREG) return launch_v<GRP_D, AM_MVREG>(ctx, L, B, R, S, next, tier);
  return AM_ERR_UNSUPPORTED;
}

#if defined(AMK_PHASE_PROF) && GRP_D == 8
// experiments only: read and clear the wave kernel's phase cycle sums (the D = 8 build: C3)
extern "C" int am_debug_phase_cycles(uint64_t *out) {
  unsigned long long h[8] = {0};
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(amk_grp::amk_phase_cycles), sizeof(h)) != hipSuccess) return AM_ERR_HIP;
  for (int i = 0; i < 8; ++i) out[i] = h[i];
  const unsigned long long z[8] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(amk_grp::amk_phase_cycles), z, sizeof(z)) == hipSuccess ? AM_OK : AM_ERR_HIP;
}
#endif
