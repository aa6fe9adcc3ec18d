"""Read batching at the caller.

The reference fans a transaction's reads out one key at a time:
clocksi_interactive_coord:execute_command(read_objects, Objects, ...)
(src/clocksi_interactive_coord.erl:732-747) maps every {Key, Type} to its partition with
log_utilities:get_key_partition/1 (src/log_utilities.erl:60-61) and sends one
async_read_data_item per key; each read server then calls materializer_vnode:read/6 for
that key (src/clocksi_readitem_server.erl:217-228, 272).  Here the same fan-out is grouped:
the objects of one partition become ONE am_materialize batch against that partition's
ops cache in HBM, and results come back in request order, as the coordinator's
return_accumulator does.  Integer keys only (get_key_partition's integer branch,
am_key_partition); every call runs the HIP library (no CPU path).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

from . import abi
from .materializer import Materializer, Store
from .oplog import HostLog, Op, Read


class PartitionedReader:
    """One node's partitions (vnodes), each with its own ops cache (am_store) on the GPU."""

    def __init__(self, mat: Materializer, n_partitions: int, n_dc: int,
                 objects: Dict[int, Tuple[int, Sequence[Op]]]):
        """objects: Key -> (Type, committed ops oldest -> newest) -- the ops caches to load."""
        self.mat, self.n_partitions, self.n_dc = mat, n_partitions, n_dc
        L = abi.lib()
        per_part: List[List[int]] = [[] for _ in range(n_partitions)]
        for key in sorted(objects):
            per_part[L.am_key_partition(key, n_partitions)].append(key)
        self.where: Dict[int, Tuple[int, int]] = {}
        self.stores: List[Optional[Store]] = []
        for p, keys in enumerate(per_part):
            for i, key in enumerate(keys):
                self.where[key] = (p, i)
            if keys:
                log = HostLog(n_dc, [list(objects[k][1]) for k in keys], key_types=[objects[k][0] for k in keys])
                self.stores.append(mat.store(log))
            else:
                self.stores.append(None)

    def partition_of(self, key: int) -> int:
        return abi.lib().am_key_partition(key, self.n_partitions)

    def read_objects(self, objects: Sequence[Tuple[int, int]], snapshot_time: Dict[int, int],
                     txid: Optional[int] = None) -> list:
        """read_objects for one transaction: [(Key, Type)] at one snapshot time ->
        per object ('ok', Value, NewLastOp, LastOpCt, IsNewSS, Count, flags) or ('error', status),
        in request order.  A key with no ops cache entry reads as an empty log (new())."""
        groups: Dict[int, List[Tuple[int, int, int]]] = {}
        out: list = [None] * len(objects)
        for pos, (key, type_) in enumerate(objects):
            if key not in self.where:
                raise KeyError(f"key {key} has no ops cache entry on this node")
            p, local = self.where[key]
            groups.setdefault(p, []).append((pos, local, type_))
        for p, items in groups.items():
            reads = [Read(local, type_, dict(snapshot_time), txid) for _pos, local, type_ in items]
            hb = self.mat.read_batch(self.stores[p], reads)
            for j, (pos, _local, _t) in enumerate(items):
                out[pos] = hb.result(j)
        return out

    def close(self):
        for s in self.stores:
            if s is not None:
                s.close()
        self.stores = []
