"""Full-population parity of the bench configs (SURVEY.md 8(a) "per-key output contract",
src/clocksi_materializer.erl:89-101): EVERY read of bench.py's step -- one batch over every
key of the GPU at the q = 0.75 clock, C2 1M LWW keys x 256 ops, C3 1M AW keys x 1024 ops,
C4 8M mixed keys x 16 ops, C5 2M Zipf MV / bounded-counter keys -- against the C oracle over
the host-regenerated log (tests/fullpop.py), every output column compared.  The C4 case then
plants a one-op change in the device log and checks that exactly the changed key is flagged."""
import ctypes

import numpy as np
import pytest
import torch

import bench
from antidote_amd import abi, synth
from antidote_amd.devbatch import DeviceReads, materialize
from tests import fullpop

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mat():
    from antidote_amd.materializer import Materializer
    m = Materializer(0)
    yield m
    m.close()


def _device_read(mat, dlog, p, kt, cfg, clock):
    type_ = cfg["type"]
    mixed = type_ not in range(1, 6)
    dr = DeviceReads(p.n_keys, p.n_dc, 0 if mixed else type_, clock, set_cap=max(cfg["set_cap"], 1),
                     types=torch.from_numpy(kt.copy()).cuda() if mixed else None)
    torch.cuda.synchronize()
    materialize(mat, dlog, dr)
    mat.sync()
    dev = fullpop.device_results(dr)
    del dr
    return dev


@pytest.mark.timeout(900)
@pytest.mark.parametrize("cfg_name,escape", [("c2", 0.0), ("c3", 0.0), ("c4", 0.0), ("c5", 0.0), ("c2", 0.1),
                                             ("c3", 0.1), ("c4", 0.1), ("c5", 0.1)],
                         ids=["c2", "c3", "c4", "c5", "c2-esc10", "c3-esc10", "c4-esc10", "c5-esc10"])
def test_fullpop_config(mat, cfg_name, escape):
    """escape: the fraction of ops with one remote DC's snapshot entry 2^33 us behind (bench.py
    --escape), which the packed view escapes: their inclusion comes from the full columns."""
    cfg = dict(bench.CONFIGS[cfg_name], escape=escape)
    p = bench.synth_params(cfg)
    st = mat.synth_store(p)
    try:
        st.index(abi.AM_INDEX_NONE)  # the bench headline's store: every op streamed
        dlog = st.device_log()
        ko, kt = bench.key_columns(mat, dlog, p.n_keys)
        lens = np.diff(ko.astype(np.int64))
        clock = synth.read_clock(p, bench.Q)
        cap = max(cfg["set_cap"], 1)
        dev = _device_read(mat, dlog, p, kt, cfg, clock)
        dev["_key_type"] = kt
        n, ops, bad = fullpop.full_parity(p, clock, cap, dev, lens)
        assert n == p.n_keys and ops == int(ko[-1])
        assert len(bad) == 0, (cfg_name, len(bad), bad[:16].tolist())
        print(f"{cfg_name} escape {escape}: {n} reads / {ops} ops bit-exact")

        if cfg_name == "c4" and not escape:
            # a planted one-op change: the oldest op of a PN key leaves the snapshot (its DC-0
            # packed entry, and its lag view commit entry where the store has one, above every
            # threshold); the comparator must flag that key alone
            k = int(np.nonzero((kt == abi.AM_PN) & (dev["count"] > 0) & (lens > 0))[0][1000])
            pos = int(ko[k])
            stride = dlog.snap_stride or dlog.n_ops
            v = np.array([0xFFFFFFFE], np.uint32)
            abi.check(mat.L.am_memcpy_h2d(mat.ctx, ctypes.c_void_p(dlog.pk_vc + 4 * (0 * stride + pos)),
                                          v.ctypes.data, 4), "am_memcpy_h2d")
            if dlog.lag_ct:
                abi.check(mat.L.am_memcpy_h2d(mat.ctx, ctypes.c_void_p(dlog.lag_ct + 4 * pos), v.ctypes.data, 4),
                          "am_memcpy_h2d")
            mat.sync()
            dev2 = _device_read(mat, dlog, p, kt, cfg, clock)
            k0 = max(0, k - 100)
            ref = fullpop.oracle_chunk(p, k0, 200, clock, cap)
            got = fullpop.compare_chunk(dev2, ref, k0, 200) + k0
            assert got.tolist() == [k], got.tolist()
            assert int(dev2["count"][k]) == int(dev["count"][k]) - 1
    finally:
        st.close()
        torch.cuda.empty_cache()
