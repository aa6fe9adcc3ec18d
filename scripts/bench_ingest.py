#!/usr/bin/env python3
"""In-place op-cache ingestion (am_store_apply) against the whole-store rebuild (am_store_update)
on a C3-shaped ops cache (add-wins set, D = 8, 1024 ops per key).

materializer_vnode:op_insert_gc/3 appends one op to one key in O(1) (src/materializer_vnode.erl:
622-647).  Here an insert batch touching a fraction f of the keys (one op each) is applied two
ways to the same store:
  * rebuild: am_store_update with the new ops as CSR over every key -- every column, the packed
    view and the token-group view of the whole store are rewritten (O(store));
  * in place: am_store_apply on the store with room for appends (am_store_reserve once) -- only
    the touched keys are rebuilt and written back into their room (O(touched keys' ops)).
Prints one JSON line per fraction: wall ms per batch (median) with the zone index kept current
and without one, touched keys, and the rebuild's ms for the same batch.  The appended op of a touched key is a copy of one of its own
log's ops (a valid effect of its type)."""
import argparse
import json
import os
import random
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402

from antidote_amd import abi, synth  # noqa: E402
from antidote_amd.materializer import Materializer  # noqa: E402
from antidote_amd.oplog import HostLog  # noqa: E402


def new_ops_log(src: HostLog, n: int, pick):
    """A host log of n keys, key i holding one op: op pick(i) of the source log."""
    idx = np.asarray([pick(i) for i in range(n)], np.int64)
    log = HostLog.__new__(HostLog)
    log.n_dc, log.n_keys, log.n_ops, log.has_var = src.n_dc, n, n, src.has_var
    log.key_off = np.arange(n + 1, dtype=np.uint64)
    log.key_type = np.full(max(n, 1), src.key_type[0], np.uint8)
    log.key_flags = log.key_id_base = log.snap_pres = log.op_txid = log.op_id = None
    log.op_meta = src.op_meta[idx].copy()
    log.commit_time = src.commit_time[idx].copy()
    log.snap_vc = np.ascontiguousarray(src.snap_vc[:, idx])
    log.p0, log.p1 = src.p0[idx].copy(), src.p1[idx].copy()
    if src.has_var:
        lens = (src.var_off[idx + 1] - src.var_off[idx]).astype(np.uint64)
        log.var_off = np.concatenate([np.zeros(1, np.uint64), np.cumsum(lens, dtype=np.uint64)])
        log.var_data = np.concatenate([src.var_data[int(src.var_off[p]):int(src.var_off[p + 1])] for p in idx]
                                      + [np.zeros(1, np.uint64)]).astype(np.uint64)
        log.n_var = int(log.var_off[-1])
    else:
        log.var_off = log.var_data = None
        log.n_var = 0
    return log


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", type=int, default=1 << 18)
    ap.add_argument("--ops", type=int, default=1024)
    ap.add_argument("--fractions", default="0.001,0.01,0.1")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--rebuild-steps", type=int, default=2)
    args = ap.parse_args()
    n_dc = 8
    mat = Materializer(0)
    p = synth.params(args.keys, n_dc, abi.AM_AWSET, ops_per_key=args.ops)
    base = mat.synth_store(p)
    src = synth.host_log(p, 0, 256)  # op donors
    t0 = time.perf_counter()
    room = base.reserve()
    mat.sync()
    reserve_ms = (time.perf_counter() - t0) * 1e3
    rng = random.Random(11)
    levels = {"summaries": abi.AM_INDEX_SUMMARIES, "none": abi.AM_INDEX_NONE}
    for f in [float(x) for x in args.fractions.split(",")]:
        m = max(1, int(args.keys * f))
        times = {}  # in-place ms per zone-index level: the maintained index's cost (k_writeback)
        for name, level in levels.items():
            room.index(level)
            times[name] = []
            for step in range(args.steps + 1):
                keys = sorted(rng.sample(range(args.keys), m))
                log = new_ops_log(src, m, lambda i: int(src.key_off[i % 256]) + rng.randrange(args.ops))
                t0 = time.perf_counter()
                ok, _ = room.apply(keys, new_log=log)
                dt = (time.perf_counter() - t0) * 1e3
                assert ok, "a touched key outgrew its room"
                if step:
                    times[name].append(dt)
        rb = []
        for _ in range(args.rebuild_steps):
            keys = sorted(rng.sample(range(args.keys), m))
            part = new_ops_log(src, m, lambda i: int(src.key_off[i % 256]))
            full = HostLog.__new__(HostLog)
            full.__dict__.update(part.__dict__)
            full.n_keys = args.keys
            ko = np.zeros(args.keys + 1, np.uint64)
            cnt = np.zeros(args.keys, np.uint64)
            cnt[keys] = 1
            ko[1:] = np.cumsum(cnt)
            full.key_off = ko
            full.key_type = np.full(args.keys, abi.AM_AWSET, np.uint8)
            t0 = time.perf_counter()
            s1, _ = base.update(new_log=full)
            mat.sync()
            rb.append((time.perf_counter() - t0) * 1e3)
            s1.close()
        print(json.dumps({"metric": "op-cache ingestion: one insert batch (1 op per touched key), wall ms",
                          "touched_keys": m, "fraction": f, "in_place_ms": float(np.median(times["summaries"])),
                          "in_place_ms_no_index": float(np.median(times["none"])),
                          "rebuild_ms": float(np.median(rb)), "reserve_ms_once": reserve_ms,
                          "config": {"workload": f"c3-shaped ops cache: add-wins set, {args.keys} keys x {args.ops} "
                                                 f"ops, D={n_dc}", "in_place": "am_store_apply (zone index at summaries, kept current by k_writeback; "
                                                 "in_place_ms_no_index: without an index)",
                                     "rebuild": "am_store_update (new ops as CSR over every key)"}}), flush=True)
    room.close()
    base.close()
    mat.close()


if __name__ == "__main__":
    main()
