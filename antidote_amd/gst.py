"""Global stable time (GST) across GPUs: the node-level exchange of meta_data_sender
(src/meta_data_sender.erl:232-255) as one element-wise MIN all-reduce.

Encoding (shared with am_gst_local_min / am_gst_allreduce / am_gst_finalize in
antidote_amd/csrc/am_gst.hip): a node dict {DcIdx: Time} becomes n_dc+1 u64 lanes, DC
absent -> 2^64-1 (min-neutral: get_min_time only mins over dicts that hold the DC,
src/stable_time_functions.erl:51-85), lane n_dc = 1 for a defined dict and 0 for
'undefined' (min = "some node undefined", which zeroes every merged DC).

On GPUs the all-reduce is RCCL (am_gst_allreduce).  `allreduce_lanes` is the same
reduction over any torch.distributed group (gloo on the CPU control plane), used by the
multi-process tests; unsigned order is mapped onto torch's signed MIN by flipping the
sign bit.
"""
from __future__ import annotations

from typing import Dict, Optional, Sequence

import numpy as np

ABSENT = np.uint64(0xFFFFFFFFFFFFFFFF)
SIGN = np.uint64(0x8000000000000000)
UNDEFINED = None


def encode_node(d: Optional[Dict[int, int]], n_dc: int) -> np.ndarray:
    lanes = np.full(n_dc + 1, ABSENT, np.uint64)
    if d is UNDEFINED:
        lanes[n_dc] = 0
        return lanes
    for dc, t in d.items():
        if not 0 <= int(t) < 2**64 - 1:
            raise ValueError("clock values must be < 2^64-1")
        lanes[dc] = t
    lanes[n_dc] = 1
    return lanes


def decode(lanes: np.ndarray, n_dc: int) -> Dict[int, int]:
    """Merged lanes -> get_min_time's dict (undefined => every present DC is 0)."""
    undef = int(lanes[n_dc]) == 0
    return {d: (0 if undef else int(lanes[d])) for d in range(n_dc) if lanes[d] != ABSENT}


def allreduce_lanes(lanes: np.ndarray, group=None) -> np.ndarray:
    import torch
    import torch.distributed as dist
    t = torch.from_numpy((lanes ^ SIGN).view(np.int64).copy())
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return t.numpy().view(np.uint64) ^ SIGN


def owned_partitions(n_partitions: int, rank: int, world: int) -> Sequence[int]:
    """riak_core partition p is served by GPU p mod N (one process per GPU)."""
    return [p for p in range(n_partitions) if p % world == rank]


# ---- the C-ABI host twins of the device GST path (am_gst_*_host, one source with the kernels)
def local_min_host(table: Dict[int, Optional[Dict[int, int]]], n_dc: int) -> np.ndarray:
    """am_gst_local_min_host over a node's partitions {partition: dict | UNDEFINED} -> lanes."""
    from . import abi
    parts = sorted(table)
    vc = np.zeros((max(len(parts), 1), n_dc), np.uint64)
    pres = np.zeros(max(len(parts), 1), np.uint32)
    undef = np.zeros(max(len(parts), 1), np.uint8)
    for i, p in enumerate(parts):
        d = table[p]
        if d is UNDEFINED or d == "undefined":  # None, or the oracle's atom
            undef[i] = 1
            continue
        for dc, t in d.items():
            vc[i, dc] = t
            pres[i] |= np.uint32(1 << dc)
    lanes = np.zeros(n_dc + 1, np.uint64)
    abi.check(abi.lib().am_gst_local_min_host(n_dc, len(parts), vc.ctypes.data, pres.ctypes.data, undef.ctypes.data,
                                              lanes.ctypes.data), "am_gst_local_min_host")
    return lanes


def merge_host(lanes: np.ndarray, into: np.ndarray, n_dc: int) -> np.ndarray:
    """am_gst_merge_lanes_host: the all-reduce's element-wise min of two nodes' lanes."""
    from . import abi
    out = np.ascontiguousarray(into, np.uint64).copy()
    a = np.ascontiguousarray(lanes, np.uint64)
    abi.check(abi.lib().am_gst_merge_lanes_host(n_dc, a.ctypes.data, out.ctypes.data), "am_gst_merge_lanes_host")
    return out


class StableHost:
    """meta_data_sender's stable state for one node (am_gst_finalize_host): the monotone update
    of the merged lanes, and the snapshot a reader gets (gr: min broadcast to every DC)."""

    def __init__(self, n_dc: int):
        self.n_dc = n_dc
        self.last_vc = np.zeros(n_dc, np.uint64)
        self.last_pres = np.zeros(1, np.uint32)

    def update(self, lanes: np.ndarray, gr: bool = False):
        from . import abi
        out = np.zeros(self.n_dc, np.uint64)
        pres = np.zeros(1, np.uint32)
        ch = np.zeros(1, np.uint8)
        ln = np.ascontiguousarray(lanes, np.uint64)
        abi.check(abi.lib().am_gst_finalize_host(self.n_dc, ln.ctypes.data, self.last_vc.ctypes.data,
                                                 self.last_pres.ctypes.data, 1 if gr else 0, out.ctypes.data,
                                                 pres.ctypes.data, ch.ctypes.data), "am_gst_finalize_host")
        snap = {d: int(out[d]) for d in range(self.n_dc) if (int(pres[0]) >> d) & 1}
        return bool(ch[0]), snap
