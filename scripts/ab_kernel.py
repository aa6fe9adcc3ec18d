"""A/B the materialize kernel variants on one GPU, interleaved in one process
(cdna_hip_programming.md 5.4 rule 24).  Usage: python scripts/ab_kernel.py [config] [rounds]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import bench
from antidote_amd import abi
from antidote_amd.devbatch import DeviceReads, materialize
from antidote_amd.materializer import Materializer

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 10
variants = (sys.argv[3] if len(sys.argv) > 3 else "stream,scalar").split(",")
type_, n_dc, n_keys, n_ops, q = bench.CONFIGS[cfg]
mat = Materializer(0)
p = bench.synth_params(type_, n_dc, n_keys, n_ops, 0)
st = mat.synth_store(p)
dlog = st.device_log()
clock = (ctypes.c_uint64 * n_dc)()
abi.lib().am_synth_read_clock(ctypes.byref(p), q, clock)
reads = DeviceReads(n_keys, n_dc, type_, list(clock))
torch.cuda.synchronize()
alg = n_keys * (n_ops * bench.bytes_per_op(type_, n_dc, False) + bench.bytes_per_key(type_, n_dc))  # full-view bytes
times = {v: [] for v in variants}
ref = None
for rd in range(rounds):
    for v in variants:
        # variant = "label" or "label:ENV=VAL;ENV=VAL"
        label, _, envs = v.partition(":")
        for k in ("AM_KERNEL", "AM_PACKED"):
            os.environ.pop(k, None)
        os.environ["AM_KERNEL"] = label
        for kv in filter(None, envs.split(";")):
            k, _, val = kv.partition("=")
            os.environ[k] = val
        materialize(mat, dlog, reads)  # warm
        abi.lib().am_timer_start(mat.ctx)
        for _ in range(5):
            materialize(mat, dlog, reads)
        ms = ctypes.c_float()
        abi.lib().am_timer_stop(mat.ctx, ctypes.byref(ms))
        times[v].append(ms.value / 5)
        if rd == 0:
            h = reads.host()
            sig = [h[k].tobytes() for k in ("status", "new_last_op", "last_ct", "count", "v0", "v1", "vflag")]
            if ref is None:
                ref = sig
            else:
                assert sig == ref, f"variant {v} differs"
for v in variants:
    t = np.array(times[v])
    print(f"{cfg} {v:8s} median {np.median(t):.3f} ms  min {t.min():.3f}  -> {alg / (np.median(t) * 1e-3) / 1e9:.0f} GB/s "
          f"({alg / (np.median(t) * 1e-3) / 8e12 * 100:.1f}% of 8 TB/s)")
