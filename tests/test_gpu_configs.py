"""BASELINE.json config shapes (C1..C5) at parity-test scale: the device generator's
log materialized by the HIP kernels, checked against the oracle on the bit-identical
host-regenerated log (sampled keys), fresh reads at two snapshot quantiles."""
import numpy as np
import pytest
import torch

from antidote_amd import abi, synth
from antidote_amd.devbatch import DeviceReads, materialize
from antidote_amd.oplog import HostBatch, Read
from oracle import amo
from tests import randlog

pytestmark = pytest.mark.gpu

SHAPES = {
    # name: synth.params kwargs (parity-test scale of BASELINE.json configs)
    "c1_pn": dict(n_keys=10000, n_dc=1, type_=abi.AM_PN, ops_per_key=64),
    "c2_lww": dict(n_keys=8192, n_dc=3, type_=abi.AM_LWW, ops_per_key=256),
    "c3_awset": dict(n_keys=1500, n_dc=8, type_=abi.AM_AWSET, ops_per_key=1024, universe=64),
    "c4_mixed": dict(n_keys=20000, n_dc=3, type_=0, ops_per_key=16),
    "c5_mv_bc_zipf": dict(n_keys=20000, n_dc=16, type_=abi.AM_SYNTH_MV_BC, zipf=1.1, total_ops=300000,
                          hot_cap=900),
    # hot keys far beyond the LDS tier (the big-read path, am_big.hip)
    "c5_hot": dict(n_keys=3000, n_dc=16, type_=abi.AM_SYNTH_MV_BC, zipf=1.1, total_ops=400000, hot_cap=60000),
    "c3_long": dict(n_keys=24, n_dc=8, type_=abi.AM_AWSET, ops_per_key=9000, universe=64),
}


@pytest.fixture(scope="module")
def mat():
    from antidote_amd.materializer import Materializer
    m = Materializer(0)
    yield m
    m.close()


@pytest.mark.parametrize("name", sorted(SHAPES))
def test_config_shape_parity(mat, name):
    p = synth.params(**SHAPES[name])
    st = mat.synth_store(p)
    dlog = st.device_log()
    hlog = synth.host_log(p, 0, p.n_keys)
    # the device log equals the host regeneration (spot-check the columns)
    n_ops = int(hlog.n_ops)
    assert dlog.n_ops == n_ops
    assert dlog.n_var == hlog.n_var
    ktypes = hlog.key_type[:p.n_keys]
    rng = np.random.default_rng(3)
    for q in (0.5, 0.9):
        clock = synth.read_clock(p, q)
        for t in sorted(set(int(x) for x in ktypes)):
            keys = np.nonzero(ktypes == t)[0]
            kt = torch.from_numpy(keys.astype(np.int64)).cuda()
            dr = DeviceReads(len(keys), p.n_dc, t, clock, keys=kt, set_cap=128)
            torch.cuda.synchronize()
            materialize(mat, dlog, dr)
            mat.sync()
            h = dr.host()
            sample = np.sort(rng.choice(len(keys), min(200, len(keys)), replace=False))
            reads = [Read(int(keys[i]), t, {d: clock[d] for d in range(p.n_dc)}) for i in sample]
            ref = amo.materialize(hlog, HostBatch(p.n_dc, reads, randlog.caps_for(reads, p.n_dc, 128)))
            vals = dr.values(sample)
            for j, i in enumerate(sample):
                r = ref.result(j)
                assert r[0] == "ok", (name, t, r)
                assert int(h["status"][i]) == 0, (name, t, int(h["status"][i]))
                ct = None if h["last_ct_ignore"][i] else {d: int(h["last_ct"][d, i]) for d in range(p.n_dc)
                                                          if (int(h["last_ct_pres"][i]) >> d) & 1}
                got = ("ok", vals[j], int(h["new_last_op"][i]), ct, bool(h["is_new_ss"][i]), int(h["count"][i]),
                       int(h["flags"][i]))
                assert got == r, (name, t, int(keys[i]), got, r)
            assert (h["status"] == 0).all(), (name, t)
    st.close()


@pytest.mark.parametrize("name", ["c4_mixed", "c5_mv_bc_zipf", "c5_hot"])
def test_config_mixed_batch_parity(mat, name):
    """The whole store read as ONE mixed-type batch (the planner splits it on the device),
    sampled keys checked against the oracle."""
    p = synth.params(**SHAPES[name])
    st = mat.synth_store(p)
    dlog = st.device_log()
    hlog = synth.host_log(p, 0, p.n_keys)
    ktypes = hlog.key_type[:p.n_keys].copy()
    clock = synth.read_clock(p, 0.75)
    dr = DeviceReads(p.n_keys, p.n_dc, 0, clock, set_cap=128, types=torch.from_numpy(ktypes).cuda())
    torch.cuda.synchronize()
    materialize(mat, dlog, dr)
    mat.sync()
    h = dr.host()
    assert (h["status"] == 0).all(), np.unique(h["status"], return_counts=True)
    rng = np.random.default_rng(5)
    lens = np.diff(hlog.key_off.astype(np.int64))[:p.n_keys]
    hot = np.argsort(-lens)[:8]  # always include the longest logs
    sample = np.unique(np.concatenate([hot, rng.choice(p.n_keys, min(300, p.n_keys), replace=False)]))
    reads = [Read(int(k), int(ktypes[k]), {d: clock[d] for d in range(p.n_dc)}) for k in sample]
    ref = amo.materialize(hlog, HostBatch(p.n_dc, reads, randlog.caps_for(reads, p.n_dc, 128)))
    vals = dr.values(sample)
    for j, i in enumerate(sample):
        ct = None if h["last_ct_ignore"][i] else {d: int(h["last_ct"][d, i]) for d in range(p.n_dc)
                                                  if (int(h["last_ct_pres"][i]) >> d) & 1}
        got = ("ok", vals[j], int(h["new_last_op"][i]), ct, bool(h["is_new_ss"][i]), int(h["count"][i]),
               int(h["flags"][i]))
        assert got == ref.result(j), (name, int(i), int(ktypes[i]), got, ref.result(j))
    st.close()


def test_config_mixed_batch_foreign_types(mat):
    """A mixed batch over an MV + bounded-counter log whose reads also name types the log has no
    keys of (AW set, PN, LWW) or the other present type: every such read of a key with ops gets
    corrupted_ops_cache (src/clocksi_materializer.erl:190-191) -- the planner skips the chains of
    absent set types, so those statuses must come from the lane tier -- and the rest stay exact."""
    p = synth.params(**SHAPES["c5_mv_bc_zipf"])
    st = mat.synth_store(p)
    dlog = st.device_log()
    hlog = synth.host_log(p, 0, p.n_keys)
    ktypes = hlog.key_type[:p.n_keys].copy()
    lens = np.diff(hlog.key_off.astype(np.int64))[:p.n_keys]
    rtypes = ktypes.copy()
    idx = np.arange(p.n_keys)
    rtypes[idx % 7 == 3] = abi.AM_AWSET
    rtypes[idx % 11 == 5] = abi.AM_PN
    rtypes[idx % 13 == 6] = abi.AM_LWW
    swap = idx % 17 == 8  # the other present type
    rtypes[swap] = np.where(ktypes[swap] == abi.AM_MVREG, abi.AM_BCOUNTER, abi.AM_MVREG)
    clock = synth.read_clock(p, 0.75)
    dr = DeviceReads(p.n_keys, p.n_dc, 0, clock, set_cap=128, types=torch.from_numpy(rtypes).cuda())
    torch.cuda.synchronize()
    materialize(mat, dlog, dr)
    mat.sync()
    h = dr.host()
    foreign = (rtypes != ktypes) & (lens > 0)
    assert foreign.sum() > 0
    assert (h["status"][foreign] == abi.AM_ERR_CORRUPTED_OPS_CACHE).all(), \
        np.unique(h["status"][foreign], return_counts=True)
    assert (h["status"][~foreign] == 0).all(), np.unique(h["status"][~foreign], return_counts=True)
    rng = np.random.default_rng(9)
    sample = np.sort(rng.choice(np.flatnonzero(~foreign), 200, replace=False))
    reads = [Read(int(k), int(ktypes[k]), {d: clock[d] for d in range(p.n_dc)}) for k in sample]
    ref = amo.materialize(hlog, HostBatch(p.n_dc, reads, randlog.caps_for(reads, p.n_dc, 128)))
    vals = dr.values(sample)
    for j, i in enumerate(sample):
        ct = None if h["last_ct_ignore"][i] else {d: int(h["last_ct"][d, i]) for d in range(p.n_dc)
                                                  if (int(h["last_ct_pres"][i]) >> d) & 1}
        got = ("ok", vals[j], int(h["new_last_op"][i]), ct, bool(h["is_new_ss"][i]), int(h["count"][i]),
               int(h["flags"][i]))
        assert got == ref.result(j), (int(i), got, ref.result(j))
    st.close()
