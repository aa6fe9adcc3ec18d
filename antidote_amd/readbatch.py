"""Read batching at the caller.

The reference fans a transaction's reads out one key at a time:
clocksi_interactive_coord:execute_command(read_objects, Objects, ...)
(src/clocksi_interactive_coord.erl:732-747) maps every {Key, Type} to its partition with
log_utilities:get_key_partition/1 (src/log_utilities.erl:60-61) and sends one
async_read_data_item per key; each read server then calls materializer_vnode:read/6 for
that key (src/clocksi_readitem_server.erl:217-228, 272).  Here the partitions this GPU owns
share one vnode (ops cache + snapshot cache in HBM) whose key space concatenates theirs, and a
transaction's reads over all of them are ONE asynchronous C-ABI call
(am_read_objects_submit / am_ticket_wait): internal_read/7 for every object in one batch,
results in request order, as the coordinator's return_accumulator collects them.  Integer
keys (get_key_partition's integer branch, am_key_partition); every call runs the HIP library
(no CPU path).
"""
from __future__ import annotations

import ctypes
import weakref
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import abi
from .materializer import Materializer, Vnode
from .oplog import HostBatch, Op, Read


class PendingRead:
    """A submitted read_objects call (am_ticket); result() waits for it.  The worker thread
    writes into this object's host buffers until the ticket is waited on, so a PendingRead
    that is dropped (or closed by its reader) waits first."""

    def __init__(self, ticket, hb: HostBatch, keep, owner=None):
        self.ticket, self.hb, self.keep, self.rc, self.owner = ticket, hb, keep, None, owner

    def wait(self) -> int:
        if self.rc is None:
            self.rc = abi.lib().am_ticket_wait(self.ticket)
            self.ticket = None
            if self.owner is not None:
                self.owner._pending.discard(self)
        return self.rc

    def result(self) -> list:
        abi.check(self.wait(), "am_read_objects")
        return [self.hb.result(i) for i in range(self.hb.n)]

    def __del__(self):
        try:
            self.wait()
        except Exception:
            pass


class PartitionedReader:
    """One node's partitions on one GPU: a vnode over the concatenated key spaces."""

    def __init__(self, mat: Materializer, n_partitions: int, n_dc: int,
                 objects: Dict[int, Tuple[int, Sequence[Op]]]):
        """objects: Key -> (Type, committed ops oldest -> newest), inserted through
        op_insert_gc/3 (am_vnode_insert_host: ids, write-triggered GC)."""
        self.mat, self.n_partitions, self.n_dc = mat, n_partitions, n_dc
        L = abi.lib()
        per_part: List[List[int]] = [[] for _ in range(n_partitions)]
        for key in sorted(objects):
            per_part[L.am_key_partition(key, n_partitions)].append(key)
        self.where: Dict[int, Tuple[int, int]] = {}
        base = [0]
        order: List[int] = []
        for p, keys in enumerate(per_part):
            for i, key in enumerate(keys):
                self.where[key] = (p, i)
            order += keys
            base.append(base[-1] + len(keys))
        self.part_key_base = np.array(base, np.uint64)
        # submitted reads not yet waited on: close() waits for them; a dropped one waits in __del__
        self._pending = weakref.WeakSet()
        self.vnode: Vnode = mat.vnode(n_dc, max(len(order), 1))
        if order:
            self.vnode.insert([list(objects[k][1]) for k in order], [objects[k][0] for k in order])

    def partition_of(self, key: int) -> int:
        return abi.lib().am_key_partition(key, self.n_partitions)

    def submit(self, objects: Sequence[Tuple[int, int]], snapshot_time: Dict[int, int],
               txid: Optional[int] = None, set_capacity: int = 4096) -> PendingRead:
        """read_objects for one transaction, asynchronously: [(Key, Type)] at one snapshot."""
        parts = np.zeros(max(len(objects), 1), np.uint32)
        reads = []
        for i, (key, type_) in enumerate(objects):
            if key not in self.where:
                raise KeyError(f"key {key} has no ops cache entry on this node")
            p, local = self.where[key]
            parts[i] = p
            reads.append(Read(local, type_, dict(snapshot_time), txid))
        hb = HostBatch(self.n_dc, reads, [set_capacity] * len(reads))
        b, r = hb.structs()
        t = ctypes.c_void_p()
        abi.check(self.mat.L.am_read_objects_submit(self.vnode.handle, self.n_partitions, self.part_key_base.ctypes.data,
                                                    parts.ctypes.data, ctypes.byref(b), ctypes.byref(r),
                                                    ctypes.byref(t)), "am_read_objects_submit")
        pr = PendingRead(t, hb, (b, r, parts), owner=self)
        self._pending.add(pr)
        return pr

    def read_objects(self, objects: Sequence[Tuple[int, int]], snapshot_time: Dict[int, int],
                     txid: Optional[int] = None) -> list:
        """Per object ('ok', Value, NewLastOp, LastOpCt, IsNewSS, Count, flags) or
        ('error', status) -- AM_ERR_COLD_PATH when the read needs the log -- in request order."""
        return self.submit(objects, snapshot_time, txid).result()

    def close(self):
        for pr in list(self._pending):
            pr.wait()
        if self.vnode is not None:
            self.vnode.close()
            self.vnode = None
