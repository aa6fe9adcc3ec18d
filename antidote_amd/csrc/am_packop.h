// am_packop.h -- one op's entry in the time-base-relative packed view (am_op_log.key_tbase /
// .pk_vc, include/antidote_mat.h), shared by k_pack (am_pack.hip) and the log rebuild
// (am_gc.hip), which writes the view of the new log from the registers it copies ops through.
#pragma once
#include <cstdint>

#include "../../include/antidote_mat.h"

// the key's time base from its first op (commit time ct, snapshot entries s[0..nd) with
// presence pres): the smallest entry within 2^31 of ct, minus 2^30, saturating at 0.  Entries
// of later ops within [base, base + 2^32 - 2] fit; the others escape.
__device__ __forceinline__ uint64_t am_pk_base(uint64_t ct, const uint64_t *s, uint32_t nd, uint32_t pres,
                                               uint32_t dc) {
  uint64_t lo = ct;
  const uint64_t floor = ct > 0x7FFFFFFFull ? ct - 0x7FFFFFFFull : 0;
  for (uint32_t d = 0; d < nd; ++d)
    if (d != dc && ((pres >> d) & 1u) && s[d] >= floor && s[d] < lo) lo = s[d];
  return lo > 0x40000000ull ? lo - 0x40000000ull : 0;
}

// entry X of an op relative to the key base; esc when it does not fit
__device__ __forceinline__ uint32_t am_pk_rel(uint64_t base, uint64_t x, bool &esc) {
  if (x < base || x - base >= (uint64_t)AM_PK_ESC) {
    esc = true;
    return 0;
  }
  return (uint32_t)(x - base);
}

// writes the op's packed column entries (X[d] = ct at its commit DC, else snapshot entry d)
template <class SnapAt>
__device__ __forceinline__ void am_pk_write(uint32_t *pk_vc, uint64_t stride, uint64_t q, uint32_t nd, uint64_t base,
                                            uint64_t ct, uint32_t meta, SnapAt snap) {
  const uint32_t dc = AM_META_DC(meta);
  bool esc = (meta & AM_META_BAD) != 0;
  for (uint32_t d = 0; d < nd; ++d) {
    const uint32_t v = am_pk_rel(base, d == dc ? ct : snap(d), esc);
    pk_vc[(uint64_t)d * stride + q] = v;
  }
  if (esc) pk_vc[q] = AM_PK_ESC;
}
