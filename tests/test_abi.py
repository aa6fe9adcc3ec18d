"""CPU checks of the boundary: the C-ABI library loads (no GPU needed) and exports every
entry point include/antidote_mat.h declares, with the struct layouts the header defines."""
import ctypes
import os
import re
import subprocess

from antidote_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "antidote_mat.h")


def declared_functions():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\**\s*(am_[a-z_0-9]+)\s*\(", src, flags=re.M)))


def test_header_lists_functions():
    fns = declared_functions()
    assert "am_materialize" in fns and "am_gst_allreduce" in fns and len(fns) >= 25


def test_library_exports_every_declared_symbol():
    L = abi.lib()
    for fn in declared_functions():
        assert hasattr(L, fn), fn
    names = {n for n, _, _ in abi.SIGNATURES}
    assert set(declared_functions()) == names


def test_nm_dynamic_symbols():
    out = subprocess.run(["nm", "-D", "--defined-only", abi.LIB_PATH], capture_output=True, text=True, check=True).stdout
    syms = {line.split()[-1] for line in out.splitlines() if line.strip()}
    for fn in declared_functions():
        assert fn in syms, fn


def test_struct_layouts_match_header():
    """Compile a tiny C program against the header and compare sizeof/offsetof with ctypes."""
    prog = r'''
#include <stdio.h>
#include <stddef.h>
#include "antidote_mat.h"
int main(void){
 printf("%zu %zu %zu %zu %zu\n", sizeof(am_op_log), sizeof(am_values), sizeof(am_read_batch), sizeof(am_read_result), sizeof(am_synth_params));
 printf("%zu %zu %zu %zu\n", offsetof(am_op_log, key_off), offsetof(am_op_log, var_data), offsetof(am_read_batch, base), offsetof(am_read_result, value));
 return 0;}
'''
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write(prog)
        exe = os.path.join(d, "t")
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        lines = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split("\n")
    sizes = list(map(int, lines[0].split()))
    offs = list(map(int, lines[1].split()))
    assert sizes == [ctypes.sizeof(abi.am_op_log), ctypes.sizeof(abi.am_values), ctypes.sizeof(abi.am_read_batch),
                     ctypes.sizeof(abi.am_read_result), ctypes.sizeof(abi.am_synth_params)]
    assert offs == [abi.am_op_log.key_off.offset, abi.am_op_log.var_data.offset, abi.am_read_batch.base.offset,
                    abi.am_read_result.value.offset]


def test_key_partition_matches_reference_rule():
    """log_utilities:get_key_partition/1 for integer keys: abs(K) rem N (+1 as a 1-based index)."""
    from oracle import ref_materializer as R
    L = abi.lib()
    for k in [0, 1, -1, 45, -45, 2**40 + 3, -(2**63)]:
        for n in [1, 4, 16, 64]:
            assert L.am_key_partition(k, n) + 1 == R.get_partition_index(k, n)


def test_synth_host_regenerates_deterministically():
    """The counter-based generator is a pure function of (seed, key, op)."""
    import numpy as np
    from tests.test_gpu_parity import _host_log_from_synth, _synth_params
    p = _synth_params(50, 32, 3, abi.AM_LWW)
    a = _host_log_from_synth(p, 0, 50)
    b = _host_log_from_synth(p, 10, 5)
    assert (a.commit_time[10 * 32:15 * 32] == b.commit_time).all()
    assert (a.snap_vc[:, 10 * 32:15 * 32] == b.snap_vc).all()
    assert (a.p0[10 * 32:15 * 32] == b.p0).all()
    # strictly increasing commit times per key; snapshot entries causally earlier
    ct = a.commit_time.reshape(50, 32)
    assert (np.diff(ct.astype(np.int64), axis=1) > 0).all()
    dc = a.op_meta & 0x1F
    own = a.snap_vc[dc, np.arange(a.n_ops)]
    assert (own < a.commit_time).all()
    # LWW timestamps unique per key
    ts = a.p0.reshape(50, 32)
    assert all(len(set(r.tolist())) == 32 for r in ts)


def test_gc_entry_points_reject_bad_arguments_without_a_gpu():
    """am_store_update / am_snapcache_gc_threshold validate before touching the device:
    a missing context, store or output is AM_ERR_INVALID (never a silent no-op)."""
    from antidote_amd import abi
    L = abi.lib()
    out = ctypes.c_void_p()
    assert L.am_store_update(None, None, None, None, None, None, None, ctypes.byref(out)) == abi.AM_ERR_INVALID
    assert L.am_snapcache_gc_threshold(None, None, None, None, None) == abi.AM_ERR_INVALID
    assert abi.AM_OPS_THRESHOLD == 50 and abi.AM_GC_PRUNED_ALL == 1 and abi.AM_GC_TRIGGER == 2
