"""Experiments only: phase cycle breakdown of the wave-per-read group kernel (k_grp_wave) on the
C3 bench workload: --cached (read/6 through the snapshot cache; fresh reads take the split
kernels), --index (zone index on); --c4: the batch-clock lane kernel (k_lane_q) on C4.  Needs a
library built with -DAMK_PHASE_PROF (AM_LIB=...)."""
import ctypes
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from antidote_amd import abi  # noqa: E402
from antidote_amd.materializer import Materializer  # noqa: E402


def main():
    c4 = "--c4" in sys.argv
    cfg = bench.CONFIGS["c4" if c4 else "c3"]
    mat = Materializer(0)
    level = abi.AM_INDEX_SUMMARIES if "--index" in sys.argv else abi.AM_INDEX_NONE
    st = bench.Step(mat, None, cfg, 0, 1, level)
    if "--cached" in sys.argv:  # read/6 through the snapshot cache (q = 0.5 bases)
        st.populate()
        run = st.cached_read
    else:
        run = st.read
    f = abi.lib().am_debug_lane_phase_cycles if c4 else abi.lib().am_debug_phase_cycles
    f.restype, f.argtypes = ctypes.c_int, [ctypes.c_void_p]
    out = (ctypes.c_uint64 * 8)()
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    f(out)
    n = 5
    for _ in range(n):
        run()
    torch.cuda.synchronize()
    f(out)
    tot = sum(out[:6])
    names = (["quad scan", "publish", "own read", "gather", "outputs", "no-take"] if c4 else
             ["meta+inputs", "op tiles", "esc+records", "scalars", "survivors", "epilogue"])
    for i, nm in enumerate(names):
        print(f"{nm:12s} {out[i] / n / 4096 / 1e3:10.1f} kcyc/wave  {100.0 * out[i] / tot:5.1f}%")


if __name__ == "__main__":
    main()
