"""Experiments only: C4 step time in a fresh process against the same after other device
work (the bench line's secondary C4 ran 1.17 ms after C3, 1.43 ms in its own process).
Usage: c4_state_probe.py MODE...  (plain | c3first | c3keep | c3store | c3reads | torchpool | padN | heatN)"""
import ctypes
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from antidote_amd import abi  # noqa: E402
from antidote_amd.materializer import Materializer  # noqa: E402


def main():
    torch.cuda.set_device(0)
    mat = Materializer(0)
    uid = (ctypes.c_char * 128)()
    abi.check(mat.L.am_comm_unique_id(uid), "am_comm_unique_id")
    comm = ctypes.c_void_p()
    abi.check(mat.L.am_comm_init(mat.ctx, 0, 1, uid, ctypes.byref(comm)), "am_comm_init")

    def barrier():
        torch.cuda.synchronize()
        mat.sync()

    keep = []
    for mode in sys.argv[1:]:
        if mode in ("c3first", "c3keep"):
            s3 = bench.Step(mat, comm, bench.CONFIGS["c3"], 0, 1, abi.AM_INDEX_NONE)
            bench.measure(s3, "fresh", 3, 1, barrier, None)
            if mode == "c3keep":
                keep.append(s3)
            else:
                s3.close()
        elif mode == "c3store":  # the C3 store only (library allocations), kept
            keep.append(mat.synth_store(bench.synth_params(bench.CONFIGS["c3"])))
        elif mode == "c3reads":  # a C3-sized read batch only (torch allocations), kept
            c3 = bench.CONFIGS["c3"]
            keep.append(bench.DeviceReads(c3["n_keys"], c3["n_dc"], c3["type"], [1] * c3["n_dc"],
                                          set_cap=c3["set_cap"]))
        elif mode == "torchpool":
            x = torch.empty(40 << 30, dtype=torch.uint8, device="cuda")
            del x
        elif mode.startswith("heat"):  # heatN: N ms of device copies (HBM-bound) just before
            a = torch.empty(4 << 30, dtype=torch.uint8, device="cuda")
            b = torch.empty_like(a)
            t_end = time.perf_counter() + int(mode[4:]) * 1e-3
            while time.perf_counter() < t_end:
                for _ in range(20):
                    b.copy_(a)
                torch.cuda.synchronize()
            del a, b
        elif mode.startswith("pad"):  # padN: N GiB held below the C4 store
            keep.append(torch.empty(int(mode[3:]) << 30, dtype=torch.uint8, device="cuda"))
        s4 = bench.Step(mat, comm, bench.CONFIGS["c4"], 0, 1, abi.AM_INDEX_NONE)
        for rep in range(2):
            m = bench.measure(s4, "fresh", 20, 3, barrier, None)
            print(f"{mode} rep{rep}: {m['dt'] / 20 * 1e3:.3f} ms/step, kernel {m['kern_ms']:.3f} ms", flush=True)
        s4.close()
    for s in keep:
        if hasattr(s, "close"):
            s.close()
    keep.clear()
    mat.L.am_comm_destroy(comm)
    mat.close()


if __name__ == "__main__":
    main()
