"""The zone map (am_op_log.zone_vc: per 256-op block an upper bound of the ops' commit
vectors) lets a read with a cached base skip the blocks inside its base snapshot
(belongs_to_snapshot_op/3: none of their ops is a candidate).  Reads through the device
snapshot cache at rising snapshot times, against the oracle's internal_read/7; the context
counter shows blocks were skipped.  Bar: bit-exact read values and statuses."""
import ctypes
import random

import pytest

from antidote_amd import abi
from antidote_amd.oplog import HostLog, Read
from oracle import ref_materializer as R
from tests import randlog
from tests.test_gpu_snapcache import _oracle_state

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mat():
    from antidote_amd.materializer import Materializer
    m = Materializer(0)
    yield m
    m.close()


def _skipped(mat, reset=True, which=abi.AM_STAT_OPS_SKIPPED):
    v = ctypes.c_uint64()
    abi.check(mat.L.am_ctx_stat(mat.ctx, which, ctypes.byref(v), 1 if reset else 0), "am_ctx_stat")
    return v.value


@pytest.mark.parametrize("t", [abi.AM_AWSET, abi.AM_MVREG])
@pytest.mark.parametrize("n_dc", [2, 8])
def test_gpu_zone_skip_cached_reads(mat, t, n_dc):
    rng = random.Random(4400 + 31 * t + n_dc)
    n_keys = 24
    keys = [randlog.rand_key_ops(rng, t, n_dc, rng.choice([0, 40, 300, 700, 1000])) for _ in range(n_keys)]
    types = [t] * n_keys
    log = HostLog(n_dc, keys, key_types=types)
    store = mat.store(log)
    cache = mat.snapshot_cache(store, n_keys)
    st = _oracle_state(keys, types)
    hi = [ops[-1].commit_time if ops else 20 for ops in keys]
    _skipped(mat)
    try:
        for q in (0.3, 0.55, 0.8, 1.0, 1.2):
            reads = []
            for k in range(n_keys):
                c = int(10 + (hi[k] - 10) * q)
                reads.append(Read(k, t, {d: c + rng.randint(0, 3) for d in range(n_dc)}))
            got = cache.read(reads, set_capacity=[4096] * n_keys)
            for i, rd in enumerate(reads):
                try:
                    ref = R.internal_read(rd.key, rd.type, dict(rd.clock), R.IGNORE, False, st)
                except R.LogColdPath:
                    ref = ("cold",)
                g = got.result(i)
                if ref[0] == "cold":
                    assert g == ("error", abi.AM_ERR_COLD_PATH), (q, rd.key, g)
                elif ref[0] == "error":
                    assert g[0] == "error", (q, rd.key, g, ref)
                else:
                    assert g[0] == "ok" and g[1] == randlog.canon_state(t, ref[1]), (q, rd.key, g, ref)
        assert _skipped(mat) > 0  # the later rounds' bases cover whole blocks
    finally:
        cache.close()
        store.close()


@pytest.mark.parametrize("t", [abi.AM_AWSET, abi.AM_MVREG])
def test_gpu_zone_fresh_exact_blocks(mat, t):
    """Fresh reads at one batch clock (the bench's step): an aligned 256-op block that is EXACT
    (one key's ops, all in the packed view) and inside the clock is included whole from its
    zone -- bits, count and LastOpCt maxima -- without streaming its commit vectors, and the
    leading such blocks' born / killed groups come from their group summaries (zone_gsum)
    without streaming their records.  Device
    generated 1024-op keys (aligned blocks), sampled keys against the oracle on the host
    regeneration; the context counter shows blocks were taken from their zones."""
    import numpy as np
    import torch
    from antidote_amd import synth
    from antidote_amd.devbatch import DeviceReads, materialize
    from antidote_amd.oplog import HostBatch
    from oracle import amo
    kw = dict(n_keys=400, n_dc=8, type_=t, ops_per_key=1024)
    if t == abi.AM_AWSET:
        kw["universe"] = 64
    p = synth.params(**kw)
    st = mat.synth_store(p)
    dlog = st.device_log()
    hlog = synth.host_log(p, 0, p.n_keys)
    rng = np.random.default_rng(5)
    try:
        for q in (0.3, 0.75, 1.0):
            clock = synth.read_clock(p, q)
            dr = DeviceReads(p.n_keys, p.n_dc, t, clock, set_cap=1100)
            torch.cuda.synchronize()
            _skipped(mat)
            _skipped(mat, which=abi.AM_STAT_RECS_SKIPPED)
            materialize(mat, dlog, dr)
            mat.sync()
            skipped = _skipped(mat)
            rskipped = _skipped(mat, which=abi.AM_STAT_RECS_SKIPPED)
            h = dr.host()
            sample = np.sort(rng.choice(p.n_keys, 60, replace=False))
            reads = [Read(int(k), t, {d: clock[d] for d in range(p.n_dc)}) for k in sample]
            ref = amo.materialize(hlog, HostBatch(p.n_dc, reads, [1100] * len(reads)))
            vals = dr.values(sample)
            for j, k in enumerate(sample):
                ct = None if h["last_ct_ignore"][k] else {d: int(h["last_ct"][d, k]) for d in range(p.n_dc)
                                                          if (int(h["last_ct_pres"][k]) >> d) & 1}
                got = ("ok", vals[j], int(h["new_last_op"][k]), ct, bool(h["is_new_ss"][k]), int(h["count"][k]),
                       int(h["flags"][k]))
                assert got == ref.result(j), (q, int(k))
            if q >= 0.75:
                assert skipped > 0  # the clock covers whole blocks
                assert rskipped > 0  # their records came from the zones' group summaries
    finally:
        st.close()


@pytest.mark.parametrize("t", [abi.AM_AWSET, abi.AM_MVREG])
def test_gpu_zone_cached_aligned_blocks(mat, t):
    """Reads through the snapshot cache (read/6, the bench's cached mode) over device-generated
    1024-op keys (aligned, exact blocks): the cache holds each key's q = 0.5 snapshot, the reads
    come at q = 0.75, so the blocks inside the base are skipped (their commit vectors, and the
    records of the leading ones) and the others streamed.
    Sampled keys against the oracle's materialize/4 with the q = 0.5 result as the base; the
    counter shows skipped ops."""
    import numpy as np
    import torch
    from antidote_amd import synth
    from antidote_amd.devbatch import DeviceReads
    from antidote_amd.oplog import HostBatch
    from oracle import amo
    kw = dict(n_keys=400, n_dc=8, type_=t, ops_per_key=1024)
    if t == abi.AM_AWSET:
        kw["universe"] = 64
    p = synth.params(**kw)
    st = mat.synth_store(p)
    dlog = st.device_log()
    hlog = synth.host_log(p, 0, p.n_keys)
    half, clock = synth.read_clock(p, 0.5), synth.read_clock(p, 0.75)
    pre = DeviceReads(p.n_keys, p.n_dc, t, half, set_cap=1100)
    dr = DeviceReads(p.n_keys, p.n_dc, t, clock, set_cap=1100)
    h = ctypes.c_void_p()
    abi.check(mat.L.am_snapcache_create(mat.ctx, p.n_dc, p.n_keys, ctypes.byref(h)), "am_snapcache_create")
    try:
        b, r = pre.structs()
        abi.check(mat.L.am_snapcache_read(mat.ctx, h, ctypes.byref(dlog), ctypes.byref(b), ctypes.byref(r)), "populate")
        torch.cuda.synchronize()
        _skipped(mat)
        _skipped(mat, which=abi.AM_STAT_RECS_SKIPPED)
        b, r = dr.structs()
        abi.check(mat.L.am_snapcache_read(mat.ctx, h, ctypes.byref(dlog), ctypes.byref(b), ctypes.byref(r)), "read")
        mat.sync()
        skipped = _skipped(mat)
        rskipped = _skipped(mat, which=abi.AM_STAT_RECS_SKIPPED)
        got_h = dr.host()
        sample = np.sort(np.random.default_rng(7).choice(p.n_keys, 60, replace=False))
        caps = [1100] * len(sample)
        s = hlog.as_struct()
        h0 = HostBatch(p.n_dc, [Read(int(k), t, {d: half[d] for d in range(p.n_dc)}) for k in sample], caps)
        b0, r0 = h0.structs()
        amo.lib().amo_materialize_range(ctypes.byref(s), ctypes.byref(b0), 0, len(sample), ctypes.byref(r0))
        assert (h0.status[:len(sample)] == 0).all()
        hb = HostBatch(p.n_dc, [Read(int(k), t, {d: clock[d] for d in range(p.n_dc)}) for k in sample], caps)
        hb.base_ignore[:] = h0.last_ct_ignore
        hb.base_vc[:] = h0.last_ct
        hb.base_pres[:] = h0.last_ct_pres
        hb.base_last_op[:] = h0.new_last_op
        hb.b_v0[:], hb.b_v1[:], hb.b_vflag[:] = h0.v0, h0.v1, h0.vflag
        hb.b_set_off, hb.b_set_len, hb.b_set_a, hb.b_set_b = h0.o_set_off, h0.o_set_len, h0.o_set_a, h0.o_set_b
        hb._h0 = h0
        b1, r1 = hb.structs()
        amo.lib().amo_materialize_range(ctypes.byref(s), ctypes.byref(b1), 0, len(sample), ctypes.byref(r1))
        vals = dr.values(sample)
        for j, k in enumerate(sample):
            ct = None if got_h["last_ct_ignore"][k] else {d: int(got_h["last_ct"][d, k]) for d in range(p.n_dc)
                                                          if (int(got_h["last_ct_pres"][k]) >> d) & 1}
            got = ("ok", vals[j], int(got_h["new_last_op"][k]), ct, bool(got_h["is_new_ss"][k]),
                   int(got_h["count"][k]), int(got_h["flags"][k]))
            assert got == hb.result(j), (int(k), got, hb.result(j))
        assert skipped > 0
        assert rskipped > 0  # the records of the leading blocks inside the base were not streamed
    finally:
        abi.check(mat.L.am_snapcache_destroy(h), "am_snapcache_destroy")
        st.close()
