#!/usr/bin/env python3
"""Experiments only: token-group and record counts per key of a config's synthetic store
(first 8192 keys): python scripts/grp_stats.py c3"""
import ctypes
import sys

import numpy as np

sys.path.insert(0, ".")
import bench  # noqa: E402
from antidote_amd import abi  # noqa: E402
from antidote_amd.materializer import Materializer  # noqa: E402


def d2h(mat, ptr, n, dt):
    a = np.zeros(n, dtype=dt)
    abi.check(mat.L.am_memcpy_d2h(mat.ctx, a.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(ptr), a.nbytes), "d2h")
    return a


def main():
    cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c3"]
    mat = Materializer(0)
    p = bench.synth_params(cfg)
    p.n_keys = min(p.n_keys, 8192)
    st = mat.synth_store(p)
    L = st.device_log()
    n = L.n_keys
    ng = d2h(mat, L.key_ngrp, n, np.uint32) & 0x7FFFFFFF
    ko = d2h(mat, L.key_off, n + 1, np.uint64)
    ro = d2h(mat, L.rec_key_off, n + 1, np.uint64)
    ops, rec = np.diff(ko), np.diff(ro)
    print("keys", n, "ops/key mean", ops.mean(), "groups/key mean/max", ng.mean(), ng.max(),
          "records/key mean", rec.mean(), "records/op", rec.sum() / max(ops.sum(), 1))
    print("group percentiles", np.percentile(ng, [10, 50, 90, 99]))
    st.close()
    mat.close()


if __name__ == "__main__":
    main()
