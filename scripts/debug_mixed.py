"""Experiments only: every read of a mixed-type batch over a test-shape store against the C
oracle (tests/fullpop.py), the mismatching reads listed with their key's shape.
   python scripts/debug_mixed.py c5_hot [reps]"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from antidote_amd import abi, synth  # noqa: E402
from antidote_amd.devbatch import DeviceReads, materialize  # noqa: E402
from antidote_amd.materializer import Materializer  # noqa: E402
from tests import fullpop  # noqa: E402
from tests.test_gpu_configs import SHAPES  # noqa: E402


def main():
    name = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    mat = Materializer(0)
    p = synth.params(**SHAPES[name])
    st = mat.synth_store(p)
    dlog = st.device_log()
    print("log: rec_g", bool(dlog.rec_g), "key_ngrp", bool(dlog.key_ngrp), "gmask", bool(dlog.gmask), "prec",
          bool(dlog.prec), "zone_vc", bool(dlog.zone_vc), flush=True)
    n = p.n_keys
    ng = np.zeros(n, np.uint32)
    abi.check(mat.L.am_memcpy_d2h(mat.ctx, ng.ctypes.data, dlog.key_ngrp, ng.nbytes), "d2h")
    ko = np.zeros(n + 1, np.uint64)
    abi.check(mat.L.am_memcpy_d2h(mat.ctx, ko.ctypes.data, dlog.key_off, ko.nbytes), "d2h")
    lens = np.diff(ko.astype(np.int64))
    hlog = synth.host_log(p, 0, n)
    kt = hlog.key_type[:n].copy()
    clock = synth.read_clock(p, 0.75)
    ref = fullpop.oracle_chunk(p, 0, n, clock, 128)
    for rep in range(reps):
        dr = DeviceReads(n, p.n_dc, 0, clock, set_cap=128, types=torch.from_numpy(kt).cuda())
        torch.cuda.synchronize()
        materialize(mat, dlog, dr)
        mat.sync()
        dev = fullpop.device_results(dr)
        bad = fullpop.compare_chunk(dev, ref, 0, n)
        print(f"rep {rep}: {len(bad)} mismatching reads of {n}", flush=True)
        for i in bad[:12]:
            g = int(ng[i])
            print(f"   read {i}: type {kt[i]} ops {lens[i]} ngrp {hex(g)} dev count {dev['count'][i]} "
                  f"ref count {ref['count'][i]} dev status {dev['status'][i]}", flush=True)
        if len(bad):
            types, cnt = np.unique(kt[bad], return_counts=True)
            print("   by type", dict(zip(types.tolist(), cnt.tolist())), "ops range", lens[bad].min(), lens[bad].max())
            print("   untouched (count 0, set_len 0):", int(((dev["count"][bad] == 0) & (ref["count"][bad] > 0)).sum()))
    st.close()
    mat.close()


if __name__ == "__main__":
    main()
