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
