"""antidote_amd -- MI355X-native batched CRDT snapshot materializer for the AntidoteDB
Cure/ClockSI read path (clocksi_materializer:materialize/4 fed by materializer_vnode's
ops and snapshot caches).  The product is libantidote_mat.so (C ABI in
include/antidote_mat.h, HIP kernels for gfx950); this package is its host mirror."""

__all__ = ["abi", "oplog", "materializer", "gst"]
