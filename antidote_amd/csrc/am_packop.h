// am_packop.h -- one op's packed streaming-view entry (am_op_log.ct_meta / .snap_delta),
// shared by k_pack (am_pack.hip) and the GC rebuild (am_gc.hip), which writes the view of
// the new log from the registers it copies the op through.
#pragma once
#include <cstdint>

#include "../../include/antidote_mat.h"

// snapshot entry s of an op relative to its commit time ct; sets esc when it does not fit
__device__ __forceinline__ int32_t am_pack_delta(uint64_t ct, uint64_t s, bool present, bool &esc) {
  if (!present) return 0;
  if (s <= ct) {
    const uint64_t diff = ct - s;
    if (diff <= 0x7FFFFFFFull) return (int32_t)diff;
  } else {
    const uint64_t diff = s - ct;
    if (diff <= 0x7FFFFFFFull) return -(int32_t)diff;
  }
  esc = true;
  return 0;
}
__device__ __forceinline__ uint64_t am_pack_ct_meta(uint64_t ct, uint32_t meta, bool esc) {
  esc = esc || ct >= AM_CT_ESC;
  return (esc ? AM_CT_ESC : ct) | ((uint64_t)meta << 56);
}
