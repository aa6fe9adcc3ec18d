"""Host mirror of the reference's materializer interface over the HIP library.

    clocksi_materializer:materialize/4  (src/clocksi_materializer.erl:82-101)
        -> Materializer.materialize(type, txid, min_snapshot_time, response)
    materializer_vnode:read/6 batched   (src/materializer_vnode.erl:96-102)
        -> Materializer.read_batch(store, reads)
    stable_time_functions:get_min_time/1 + meta_data_sender:update_stable/3
        -> antidote_amd.gst

Every call runs the HIP kernels of libantidote_mat.so (no CPU path exists).
"""
from __future__ import annotations

import ctypes
from typing import Any, Dict, List, Optional, Sequence, Tuple

from . import abi
from .oplog import HostBatch, HostLog, Op, Read

IGNORE = None


class Store:
    """A device-resident op log (one partition's ops cache in HBM)."""

    def __init__(self, mat: "Materializer", handle: ctypes.c_void_p, n_dc: int):
        self.mat, self.handle, self.n_dc = mat, handle, n_dc

    def device_log(self) -> abi.am_op_log:
        s = abi.am_op_log()
        abi.check(abi.lib().am_store_log(self.handle, ctypes.byref(s)), "am_store_log")
        return s

    def close(self):
        if self.handle:
            abi.lib().am_store_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class SnapshotCache:
    """A partition's snapshot cache on the device: reads run materializer_vnode:internal_read/7
    (src/materializer_vnode.erl:371-376) -- base from the cache, materialize/4, write-back."""

    def __init__(self, mat: "Materializer", store: "Store", n_keys: int):
        self.mat, self.store = mat, store
        self.handle = ctypes.c_void_p()
        abi.check(mat.L.am_snapcache_create(mat.ctx, store.n_dc, n_keys, ctypes.byref(self.handle)),
                  "am_snapcache_create")

    def read(self, reads: Sequence[Read]) -> HostBatch:
        """internal_read/7 (ShouldGC = false) for reads of distinct keys; read.base_* are ignored.
        Per read: ('ok', Value, ...) or ('error', AM_ERR_COLD_PATH) when the log would be read."""
        hb = HostBatch(self.store.n_dc, reads)
        b, r = hb.structs()
        abi.check(self.mat.L.am_snapcache_read_host(self.mat.ctx, self.handle, self.store.handle, ctypes.byref(b),
                                                    ctypes.byref(r)), "am_snapcache_read_host")
        return hb

    def entries(self, key: int):
        """[(clock, last_op_id, v0, v1, vflag)] newest first, or None before the key's first read."""
        import numpy as np
        nd, cap = self.store.n_dc, abi.AM_SNAPSHOT_THRESHOLD
        n = ctypes.c_uint32()
        vc = np.zeros(cap * nd, np.uint64)
        pres = np.zeros(cap, np.uint32)
        lo = np.zeros(cap, np.int64)
        v0 = np.zeros(cap, np.int64)
        v1 = np.zeros(cap, np.uint64)
        vf = np.zeros(cap, np.uint8)
        abi.check(self.mat.L.am_snapcache_get(self.mat.ctx, self.handle, key, ctypes.byref(n), vc.ctypes.data,
                                              pres.ctypes.data, lo.ctypes.data, v0.ctypes.data, v1.ctypes.data,
                                              vf.ctypes.data), "am_snapcache_get")
        if n.value == abi.AM_SNAPCACHE_ABSENT:
            return None
        out = []
        for e in range(n.value):
            clock = {d: int(vc[e * nd + d]) for d in range(nd) if (int(pres[e]) >> d) & 1}
            out.append((clock, int(lo[e]), int(v0[e]), int(v1[e]), int(vf[e])))
        return out

    def close(self):
        if self.handle:
            self.mat.L.am_snapcache_destroy(self.handle)
            self.handle = ctypes.c_void_p()


class Materializer:
    """A context on one GPU (device index = local rank)."""

    def __init__(self, device: int = 0):
        self.L = abi.lib()
        self.ctx = ctypes.c_void_p()
        abi.check(self.L.am_ctx_open(device, ctypes.byref(self.ctx)), "am_ctx_open")
        self.device = device

    def close(self):
        if self.ctx:
            self.L.am_ctx_close(self.ctx)
            self.ctx = ctypes.c_void_p()

    def sync(self):
        abi.check(self.L.am_ctx_sync(self.ctx), "am_ctx_sync")

    # ---- ops cache ----
    def store(self, log: HostLog) -> Store:
        h = ctypes.c_void_p()
        s = log.as_struct()
        abi.check(self.L.am_store_create(self.ctx, ctypes.byref(s), ctypes.byref(h)), "am_store_create")
        return Store(self, h, log.n_dc)

    def synth_store(self, params: abi.am_synth_params) -> Store:
        h = ctypes.c_void_p()
        abi.check(self.L.am_synth_store(self.ctx, ctypes.byref(params), ctypes.byref(h)), "am_synth_store")
        return Store(self, h, params.n_dc)

    # ---- the hot path ----
    def read_batch(self, store: Store, reads: Sequence[Read], set_capacity=None) -> HostBatch:
        """materializer_vnode:read/6 -> materialize/4 for a batch of keys (host memory in/out)."""
        hb = HostBatch(store.n_dc, reads, set_capacity)
        b, r = hb.structs()
        abi.check(self.L.am_materialize_host(self.ctx, store.handle, ctypes.byref(b), ctypes.byref(r)),
                  "am_materialize_host")
        return hb

    # ---- snapshot cache (materializer_vnode snapshot_cache-P in HBM) ----
    def snapshot_cache(self, store: Store, n_keys: int) -> "SnapshotCache":
        return SnapshotCache(self, store, n_keys)

    def materialize(self, type_: int, txid: Optional[int], min_snapshot_time: Dict[int, int],
                    ops_newest_first: Sequence[Tuple[int, Op]], base_clock: Optional[Dict[int, int]] = None,
                    base_last_op: int = 0, base_value: Any = None, n_dc: Optional[int] = None):
        """clocksi_materializer:materialize/4 for one key, with the #snapshot_get_response{} given
        as its parts (ops list newest first, as the reference passes it)."""
        ops = [op for _, op in reversed(list(ops_newest_first))]
        ids = [i for i, _ in reversed(list(ops_newest_first))]
        for op, i in zip(ops, ids):
            op.op_id = i
        dcs = set(min_snapshot_time) | set(base_clock or {})
        for op in ops:
            dcs |= set(op.snap) | {op.commit_dc}
        nd = n_dc or (max(dcs) + 1 if dcs else 1)
        log = HostLog(nd, [ops], key_types=[type_])
        st = self.store(log)
        try:
            hb = self.read_batch(st, [Read(0, type_, dict(min_snapshot_time), txid, base_clock, base_last_op,
                                           base_value)])
            return hb.result(0)
        finally:
            st.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
