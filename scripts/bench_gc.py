"""Op-cache GC + ingestion throughput (am_store_update) on the C2 workload.

One update = prune_ops over every key of a 1M-key x 256-op LWW log (D = 3) at a threshold
that keeps about half of each log (the synth read clock at q = 0.5), plus, with --ingest N,
N appended ops per key (op_insert_gc).  Prints one JSON line: ops in / kept / appended, wall
ms per update (device allocation + both kernels + the packed view of the new store), and
the algorithmic bytes of the compaction (thresholds resident in HBM, as the snapshot cache's are): every input column read once (op_meta 1 +
commit_time 8 + snapshot_time 8*D + p0 8 + p1 8) plus every output column written once
(the same + op_id 8).  Kernel durations come from rocprofv3 (scripts/gpu_gc.sh)."""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402

from antidote_amd import abi, synth  # noqa: E402
from antidote_amd.materializer import Materializer  # noqa: E402
from antidote_amd.oplog import HostLog  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", type=int, default=1 << 20)
    ap.add_argument("--ops", type=int, default=256)
    ap.add_argument("--q", type=float, default=0.5)
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    n_dc = 3
    mat = Materializer(0)
    p = synth.params(args.keys, n_dc, abi.AM_LWW, ops_per_key=args.ops)
    store = mat.synth_store(p)
    clock = synth.read_clock(p, args.q)
    mask = np.ones(args.keys, np.uint8)
    thr = np.repeat(np.asarray(clock, np.uint64)[:, None], args.keys, axis=1)
    pres = np.full(args.keys, (1 << n_dc) - 1, np.uint32)
    prune = (mat.device_array(mask), mat.device_array(thr), mat.device_array(pres))  # resident in HBM
    s1, _ = store.update(prune=prune)   # warm-up
    n_kept = int(s1.device_log().n_ops)
    s1.close()
    times = []
    for _ in range(args.steps):
        t0 = time.perf_counter()
        s1, _ = store.update(prune=prune)
        times.append((time.perf_counter() - t0) * 1e3)
        s1.close()
    n_in = args.keys * args.ops
    col = 1 + 8 + 8 * n_dc + 16
    alg = col * n_in + (col + 8) * n_kept
    ms = float(np.median(times))
    print(json.dumps({"metric": "op-cache GC (prune_ops) ops/s", "ops_in": n_in, "ops_kept": n_kept,
                      "ms_per_update_wall": ms, "value": n_in / ms * 1e3, "unit": "ops/s",
                      "alg_bytes_per_update": alg, "kernels": "k_upd_count + k_upd_scatter (writes the packed view of the new store too)",
                      "config": {"workload": f"c2 log: LWW, {args.keys} keys x {args.ops} ops, D={n_dc}, "
                                             f"threshold = synth clock q={args.q}"}}))
    for b in prune:
        b.free()
    store.close()
    mat.close()


if __name__ == "__main__":
    main()
