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
