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


class _DownLog:
    """A downloaded device log (Store.download: dense CSR, explicit op ids) as a host log the
    C oracle reads."""

    def __init__(self, D, n_dc):
        import numpy as np
        self.D, self.n_dc = D, n_dc
        self.snap_vc = np.ascontiguousarray(D["snap_vc"], np.uint64)
        self.n_keys = len(D["key_off"]) - 1
        self.n_ops = int(D["key_off"][-1])

    def as_struct(self):
        D = self.D
        s = abi.am_op_log()
        s.n_dc, s.n_keys, s.n_ops = self.n_dc, self.n_keys, self.n_ops
        s.n_var = len(D["var_data"]) if D["var_off"] is not None else 0
        s.snap_stride = self.snap_vc.shape[1]
        p = lambda a: None if a is None else a.ctypes.data  # noqa: E731
        s.key_off, s.key_type, s.key_flags = p(D["key_off"]), p(D["key_type"]), p(D["key_flags"])
        s.op_meta, s.commit_time, s.snap_vc, s.snap_pres = (p(D["op_meta"]), p(D["commit_time"]), p(self.snap_vc),
                                                            p(D["snap_pres"]))
        s.op_txid, s.op_id, s.p0, s.p1 = p(D["op_txid"]), p(D["op_id"]), p(D["p0"]), p(D["p1"])
        s.var_off = p(D["var_off"]) if D["var_off"] is not None and s.n_var else None
        s.var_data = p(D["var_data"]) if D["var_off"] is not None and s.n_var else None
        self._s = s
        return s


def _state_pairs(hlog, keys, t, n_dc, cap):
    """Each key's value at a clock above every op (oracle), as (a, b) pairs."""
    from antidote_amd.oplog import HostBatch
    from oracle import amo
    top = {d: (1 << 62) for d in range(n_dc)}
    hb = amo.materialize(hlog, HostBatch(n_dc, [Read(int(k), t, top) for k in keys], [cap] * len(keys)))
    out = {}
    for j, k in enumerate(keys):
        r = hb.result(j)
        assert r[0] == "ok", r
        out[int(k)] = list(r[1])
    return out


def _new_ops(rng, t, n_dc, hi, pairs, n, tok0):
    """n causally later ops of one key: AW adds of a fresh token replacing the element's live
    tokens (observe-and-replace) or removes of them; MV assigns overriding every live token."""
    from antidote_amd.oplog import Op
    ops = []
    for j in range(n):
        dc = rng.randrange(n_dc)
        snap = {d: hi[d] + (5 * j if d != dc else 0) for d in range(n_dc)}
        ct = hi[dc] + 7 + 11 * j
        tok = tok0 + j
        if t == abi.AM_AWSET:
            e = rng.randrange(64)
            live = [b for a, b in pairs if a == e]
            if live and rng.random() < 0.3:
                eff = [(e, [], live)]
                pairs = [(a, b) for a, b in pairs if a != e]
            else:
                eff = [(e, [tok], live)]
                pairs = [(a, b) for a, b in pairs if a != e] + [(e, tok)]
        else:
            v = rng.randrange(1 << 20)
            eff = ("assign", v, tok, [b for _a, b in pairs])
            pairs = [(v, tok)]
        ops.append(Op(t, dc, ct, snap, eff))
    return ops, pairs


@pytest.mark.parametrize("t", [abi.AM_AWSET, abi.AM_MVREG])
def test_gpu_zone_index_survives_apply_and_gc(mat, t):
    """The zone index under the reference's ingestion path (op_insert_gc/3 appends and
    prune_ops/2 GC, src/materializer_vnode.erl:565-647, in place through am_store_apply):
    a C3-shaped store (1024-op keys, D = 8) with room, 1-3 ops appended to 10 % of its keys and
    5 % GC-pruned; then fresh reads at q = 0.5, 0.75, 1.0 and above every op, and reads through
    the snapshot cache (q = 0.5 bases), all bit-exact against the oracle over the store's own
    downloaded log; the re-touched keys' blocks are still taken from the maintained index
    (maxima, exact marks, group summaries rewritten by k_writeback, not retired)."""
    import numpy as np
    import torch
    from antidote_amd import synth
    from antidote_amd.devbatch import DeviceReads, materialize
    from antidote_amd.oplog import HostBatch
    from oracle import amo
    n_keys, n_dc, cap = 400, 8, 1100
    kw = dict(n_keys=n_keys, n_dc=n_dc, type_=t, ops_per_key=1024)
    if t == abi.AM_AWSET:
        kw["universe"] = 64
    p = synth.params(**kw)
    base = mat.synth_store(p)
    st = base.reserve()
    base.close()
    rng = random.Random(5100 + t)
    hi = synth.read_clock(p, 1.0)
    try:
        app = sorted(rng.sample(range(n_keys), n_keys // 10))
        gc = sorted(rng.sample([k for k in range(n_keys) if k not in set(app)], n_keys // 20))
        touched = sorted(app + gc)
        pairs = _state_pairs(_DownLog(st.download(), n_dc), app, t, n_dc, cap)
        new_ops = []
        for i, k in enumerate(touched):
            if k in pairs:
                ops, _ = _new_ops(rng, t, n_dc, hi, pairs[k], rng.randint(1, 3), (1 << 60) + 8 * k)
            else:
                ops = []
            new_ops.append(ops)
        mask = np.zeros(n_keys, np.uint8)
        thr = np.zeros((n_dc, n_keys), np.uint64)
        pres = np.zeros(n_keys, np.uint32)
        q4 = synth.read_clock(p, 0.4)
        for k in gc:
            mask[k] = 1
            thr[:, k] = q4
            pres[k] = (1 << n_dc) - 1
        ok, _ = st.apply(touched, new_log=HostLog(n_dc, new_ops, key_types=[t] * len(touched)),
                         prune=(mask, thr, pres))
        assert ok
        D = st.download()
        lens = np.diff(D["key_off"].astype(np.int64))
        assert all(lens[k] == 1024 + len(o) for k, o in zip(touched, new_ops) if k in pairs)
        assert all(lens[k] < 1024 for k in gc)  # the GC pruned them
        hlog = _DownLog(D, n_dc)
        dlog = st.device_log()
        sample = sorted(set(touched) | set(int(x) for x in np.random.default_rng(3).choice(n_keys, 40, replace=False)))
        top = [h + 10_000 for h in hi]
        for q in (0.5, 0.75, 1.0, None):
            clock = top if q is None else synth.read_clock(p, q)
            dr = DeviceReads(n_keys, n_dc, t, clock, set_cap=cap)
            torch.cuda.synchronize()
            materialize(mat, dlog, dr)
            mat.sync()
            h = dr.host()
            ref = amo.materialize(hlog, HostBatch(n_dc, [Read(k, t, {d: clock[d] for d in range(n_dc)})
                                                         for k in sample], [cap] * len(sample)))
            vals = dr.values(sample)
            for j, k in enumerate(sample):
                ct = None if h["last_ct_ignore"][k] else {d: int(h["last_ct"][d, k]) for d in range(n_dc)
                                                          if (int(h["last_ct_pres"][k]) >> d) & 1}
                got = ("ok", vals[j], int(h["new_last_op"][k]), ct, bool(h["is_new_ss"][k]), int(h["count"][k]),
                       int(h["flags"][k]))
                assert got == ref.result(j), (q, k, k in app, k in gc)
        # the re-touched keys alone, above every op: their whole blocks come from the index
        kt = torch.tensor(touched, dtype=torch.int64, device="cuda")
        dr = DeviceReads(len(touched), n_dc, t, top, set_cap=cap, keys=kt)
        torch.cuda.synchronize()
        _skipped(mat)
        _skipped(mat, which=abi.AM_STAT_RECS_SKIPPED)
        materialize(mat, dlog, dr)
        mat.sync()
        skipped = _skipped(mat)
        rskipped = _skipped(mat, which=abi.AM_STAT_RECS_SKIPPED)
        assert (dr.status.cpu().numpy() == 0).all()
        # each appended AW key's four blocks stayed exact (an MV key past AM_BIG_MIN_OPS ops moves to
        # the chunked view of the big-read tier; the pruned keys' blocks are rewritten exact)
        assert skipped >= (3 * 256 * len(app) if t == abi.AM_AWSET else 256), skipped
        assert rskipped > 0
        # read/6 through the snapshot cache: q = 0.5 bases, reads at q = 0.75 and above every op
        half = synth.read_clock(p, 0.5)
        s = hlog.as_struct()
        h0 = HostBatch(n_dc, [Read(k, t, {d: half[d] for d in range(n_dc)}) for k in sample], [cap] * len(sample))
        b0, r0 = h0.structs()
        amo.lib().amo_materialize_range(ctypes.byref(s), ctypes.byref(b0), 0, len(sample), ctypes.byref(r0))
        assert (h0.status[:len(sample)] == 0).all()
        for clock in (synth.read_clock(p, 0.75), top):
            pre = DeviceReads(n_keys, n_dc, t, half, set_cap=cap)
            hc = ctypes.c_void_p()
            abi.check(mat.L.am_snapcache_create(mat.ctx, n_dc, n_keys, ctypes.byref(hc)), "am_snapcache_create")
            try:
                b, r = pre.structs()
                abi.check(mat.L.am_snapcache_read(mat.ctx, hc, ctypes.byref(dlog), ctypes.byref(b), ctypes.byref(r)),
                          "populate")
                dr = DeviceReads(n_keys, n_dc, t, clock, set_cap=cap)
                torch.cuda.synchronize()
                _skipped(mat)
                b, r = dr.structs()
                abi.check(mat.L.am_snapcache_read(mat.ctx, hc, ctypes.byref(dlog), ctypes.byref(b), ctypes.byref(r)),
                          "read")
                mat.sync()
                assert _skipped(mat) > 0
            finally:
                abi.check(mat.L.am_snapcache_destroy(hc), "am_snapcache_destroy")
            got_h = dr.host()
            hb = HostBatch(n_dc, [Read(k, t, {d: clock[d] for d in range(n_dc)}) for k in sample], [cap] * len(sample))
            hb.base_ignore[:] = h0.last_ct_ignore
            hb.base_vc[:] = h0.last_ct
            hb.base_pres[:] = h0.last_ct_pres
            hb.base_last_op[:] = h0.new_last_op
            hb.b_set_off, hb.b_set_len, hb.b_set_a, hb.b_set_b = h0.o_set_off, h0.o_set_len, h0.o_set_a, h0.o_set_b
            hb._h0 = h0
            b1, r1 = hb.structs()
            amo.lib().amo_materialize_range(ctypes.byref(s), ctypes.byref(b1), 0, len(sample), ctypes.byref(r1))
            vals = dr.values(sample)
            for j, k in enumerate(sample):
                ct = None if got_h["last_ct_ignore"][k] else {
                    d: int(got_h["last_ct"][d, k]) for d in range(n_dc) if (int(got_h["last_ct_pres"][k]) >> d) & 1}
                got = ("ok", vals[j], int(got_h["new_last_op"][k]), ct, bool(got_h["is_new_ss"][k]),
                       int(got_h["count"][k]), int(got_h["flags"][k]))
                assert got == hb.result(j), (k, k in app, k in gc, got, hb.result(j))
    finally:
        st.close()


@pytest.mark.parametrize("t", [abi.AM_AWSET, abi.AM_MVREG])
def test_gpu_zone_fresh_unaligned_keys(mat, t):
    """Fresh reads over keys whose op ranges start anywhere in a 256-slot block (a host log of
    ragged lengths): the read's tiles are aligned to the blocks, its interior exact blocks come
    from the index and the first run of them from their group summaries (a middle range of the
    record stream skipped), bit-exact against the oracle at clocks below, inside and above the
    logs; index levels NONE / ZONES / EXACT / SUMMARIES give identical results."""
    import numpy as np
    import torch
    from antidote_amd.devbatch import DeviceReads, materialize
    from antidote_amd.oplog import HostBatch
    from oracle import amo
    rng = random.Random(5300 + t)
    n_dc = 4
    keys = [randlog.rand_key_ops(rng, t, n_dc, rng.choice([3, 90, 300, 700, 1100, 1500])) for _ in range(40)]
    log = HostLog(n_dc, keys, key_types=[t] * len(keys), partial=False)
    st = mat.store(log)
    hi = max((op.commit_time for ops in keys for op in ops), default=20)
    dlog = st.device_log()
    n = len(keys)
    try:
        for q in (0.4, 0.8, 1.5):
            c = int(10 + (hi - 10) * q)
            clock = [c] * n_dc
            ref = amo.materialize(log, HostBatch(n_dc, [Read(k, t, {d: c for d in range(n_dc)}) for k in range(n)],
                                                 [4096] * n))
            outs = []
            for level in (abi.AM_INDEX_NONE, abi.AM_INDEX_ZONES, abi.AM_INDEX_EXACT, abi.AM_INDEX_SUMMARIES):
                st.index(level)
                dlog = st.device_log()
                dr = DeviceReads(n, n_dc, t, clock, set_cap=4096)
                torch.cuda.synchronize()
                _skipped(mat)
                _skipped(mat, which=abi.AM_STAT_RECS_SKIPPED)
                materialize(mat, dlog, dr)
                mat.sync()
                sk, rs = _skipped(mat), _skipped(mat, which=abi.AM_STAT_RECS_SKIPPED)
                h = dr.host()
                vals = dr.values(range(n))
                res = []
                for k in range(n):
                    ct = None if h["last_ct_ignore"][k] else {d: int(h["last_ct"][d, k]) for d in range(n_dc)
                                                              if (int(h["last_ct_pres"][k]) >> d) & 1}
                    res.append(("ok", vals[k], int(h["new_last_op"][k]), ct, bool(h["is_new_ss"][k]),
                                int(h["count"][k]), int(h["flags"][k])) if h["status"][k] == 0
                               else ("error", int(h["status"][k])))
                for k in range(n):
                    assert res[k] == ref.result(k), (q, level, k, len(keys[k]))
                outs.append(res)
                if level < abi.AM_INDEX_EXACT:
                    assert sk == 0 and rs == 0
                elif q == 1.5:
                    assert sk > 0, level
                    if level == abi.AM_INDEX_SUMMARIES:
                        assert rs > 0
    finally:
        st.close()
