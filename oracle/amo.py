"""TEST INFRASTRUCTURE ONLY: ctypes wrapper of the C oracle (oracle/am_oracle.c).

Uses the ABI struct definitions of antidote_amd.abi (data layout only); the product
never imports this module."""
import ctypes
import os
import subprocess

from antidote_amd import abi

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "_build", "libam_oracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(SO):
            build()
        L = ctypes.CDLL(SO)
        P = ctypes.POINTER
        L.amo_materialize_one.argtypes = [P(abi.am_op_log), P(abi.am_read_batch), ctypes.c_uint64,
                                          P(abi.am_read_result)]
        L.amo_materialize_range.argtypes = [P(abi.am_op_log), P(abi.am_read_batch), ctypes.c_uint64,
                                            ctypes.c_uint64, P(abi.am_read_result)]
        L.amo_gst_min.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.amo_update_stable.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_uint32]
        _lib = L
    return _lib


def materialize(log, batch, threads=1):
    """Run the oracle over every read of a HostBatch against a HostLog (host memory)."""
    s = log.as_struct()
    b, r = batch.structs()
    n = batch.n
    if threads <= 1 or n < 2 * threads:
        lib().amo_materialize_range(ctypes.byref(s), ctypes.byref(b), 0, n, ctypes.byref(r))
        return batch
    import threading
    step = (n + threads - 1) // threads
    ts = [threading.Thread(target=lib().amo_materialize_range,
                           args=(ctypes.byref(s), ctypes.byref(b), i, min(n, i + step), ctypes.byref(r)))
          for i in range(0, n, step)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return batch
