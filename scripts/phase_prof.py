"""Experiments only: phase cycle breakdown of the wave-per-read group kernel on the C3 bench
workload.  Needs a library built with -DAMK_PHASE_PROF (AM_LIB=...)."""
import ctypes
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from antidote_amd import abi, synth  # noqa: E402
from antidote_amd.materializer import Materializer  # noqa: E402


def main():
    cfg = bench.CONFIGS["c3"]
    mat = Materializer(0)
    p = bench.synth_params(cfg)
    store = mat.synth_store(p)
    if "--index" not in sys.argv:  # the bench headline's store: every op streamed
        store.index(abi.AM_INDEX_NONE)
    dlog = store.device_log()
    clock = synth.read_clock(p, 0.75)
    reads = bench.DeviceReads(cfg["n_keys"], cfg["n_dc"], cfg["type"], clock, set_cap=cfg["set_cap"])
    f = abi.lib().am_debug_phase_cycles
    f.restype, f.argtypes = ctypes.c_int, [ctypes.c_void_p]
    out = (ctypes.c_uint64 * 8)()
    for _ in range(3):
        bench.materialize(mat, dlog, reads)
    torch.cuda.synchronize()
    f(out)
    n = 5
    for _ in range(n):
        bench.materialize(mat, dlog, reads)
    torch.cuda.synchronize()
    f(out)
    tot = sum(out[:6])
    names = ["meta+inputs", "op tiles", "esc+records", "scalars", "survivors", "epilogue"]
    for i, nm in enumerate(names):
        print(f"{nm:12s} {out[i] / n / 4096 / 1e3:10.1f} kcyc/wave  {100.0 * out[i] / tot:5.1f}%")


if __name__ == "__main__":
    main()
