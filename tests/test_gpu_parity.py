"""Parity of the HIP path (libantidote_mat.so through its C ABI) against the oracle.

Bar: bit-exact -- every output column of materialize/4 (status, value, NewLastOp,
LastOpCt key set and values, IsNewSS, Count, the missing-DC log flag)."""
import random

import numpy as np
import pytest
import torch

from antidote_amd import abi
from antidote_amd.oplog import HostBatch, HostLog, Op, Read
from oracle import amo
from tests import randlog
from tests.kat_util import load
from tests.test_oracle_c import _dcmap, kat_ops, run_kat_cases

pytestmark = pytest.mark.gpu

GPU_TYPES = [abi.AM_PN, abi.AM_LWW, abi.AM_AWSET, abi.AM_MVREG, abi.AM_BCOUNTER]
SET_TYPES = (abi.AM_AWSET, abi.AM_MVREG)


@pytest.fixture(scope="module")
def mat():
    from antidote_amd.materializer import Materializer
    m = Materializer(0)
    yield m
    m.close()


KAT = load("kat_materialize.json")


@pytest.mark.parametrize("kat", KAT["materialize"], ids=lambda k: k["name"])
def test_gpu_kat(mat, kat):
    m = _dcmap(kat)
    ops = kat_ops(kat, m)
    nd = max(len(m), 1)

    def run(read):
        log = HostLog(nd, [ops], key_types=[kat["type"]])
        st = mat.store(log)
        hb = mat.read_batch(st, [read])
        st.close()
        return hb.result(0)

    run_kat_cases(kat, run)


def _batch_compare(log, reads, mat, n_dc, cap=256):
    st = mat.store(log)
    caps = [cap] * len(reads)
    got = mat.read_batch(st, reads, caps)
    st.close()
    ref = amo.materialize(log, HostBatch(n_dc, reads, caps))
    for i in range(len(reads)):
        a, b = got.result(i), ref.result(i)
        assert a == b, (i, reads[i], a, b)
    return got


@pytest.mark.parametrize("t", GPU_TYPES)
@pytest.mark.parametrize("seed", range(4))
def test_gpu_random_batches(mat, t, seed):
    """Many keys per batch: ragged lengths (0 .. 700 ops, unaligned CSR offsets, keys
    spanning several 256-op tiles), partial clocks, TxIds, cached bases, bad effects."""
    rng = random.Random(1000 + seed * 7 + t)
    n_dc = [1, 3, 5, 16][seed]
    partial = seed in (1, 3)
    keys, reads = [], []
    lens = [0, 1, 3, 17, 64, 255, 256, 257, 400] if t in SET_TYPES else [0, 1, 3, 17, 64, 255, 256, 257, 700]
    if t == abi.AM_BCOUNTER:
        n_dc = min(n_dc, 8)
    for k in range(60):
        n_ops = rng.choice(lens) if k % 5 else rng.randint(0, 40)
        ops = randlog.rand_key_ops(rng, t, n_dc, n_ops, partial=partial, txids=seed == 2,
                                   bad_rate=0.002 if seed == 3 else 0.0, t0=rng.randint(0, 100))
        keys.append(ops)
        hi = ops[-1].commit_time if ops else 50
        clock = randlog.rand_clock(rng, n_dc, 0, hi + 5, partial=partial)
        reads.append(Read(k, t, clock, rng.choice([None, 1, 3]) if seed == 2 else None))
    log = HostLog(n_dc, keys, key_types=[t] * len(keys), partial=partial or None)
    first = _batch_compare(log, reads, mat, n_dc)
    # incremental reads from the cached results (belongs_to_snapshot_op against a base clock)
    reads2 = []
    for i, r in enumerate(reads):
        res = first.result(i)
        if res[0] != "ok":
            continue
        clock2 = {d: v + rng.randint(0, 200) for d, v in r.clock.items()}
        reads2.append(Read(r.key, t, clock2, None, res[3], res[2], res[1]))
    _batch_compare(log, reads2, mat, n_dc)


def test_gpu_corrupted_and_invalid(mat):
    keys = [[Op(abi.AM_PN, 0, 5, {0: 1}, 3)], [], [Op(abi.AM_PN, 0, 5, {0: 1}, 3), Op(abi.AM_LWW, 0, 6, {0: 1}, (1, 2))]]
    log = HostLog(1, keys, key_types=[abi.AM_PN, abi.AM_LWW, abi.AM_PN])
    reads = [Read(0, abi.AM_LWW, {0: 10}), Read(1, abi.AM_LWW, {0: 10}), Read(2, abi.AM_PN, {0: 10})]
    got = _batch_compare(log, reads, mat, 1)
    assert got.result(0) == ("error", abi.AM_ERR_CORRUPTED_OPS_CACHE)
    assert got.result(1) == ("ok", (0, 0, True), 0, None, False, 0, 0)
    assert got.result(2) == ("error", abi.AM_ERR_CORRUPTED_OPS_CACHE)


def test_gpu_pn_overflow(mat):
    ops = [Op(abi.AM_PN, 0, 5 + i, {0: 1}, 2**62) for i in range(3)]
    ops2 = [Op(abi.AM_PN, 0, 5 + i, {0: 1}, v) for i, v in enumerate([2**62, 2**62, -2**62, -2**62 + 7])]
    log = HostLog(1, [ops, ops2])
    got = _batch_compare(log, [Read(0, abi.AM_PN, {0: 100}), Read(1, abi.AM_PN, {0: 100})], mat, 1)
    assert got.result(0) == ("error", abi.AM_ERR_OVERFLOW)
    assert got.result(1)[1] == 7


def _synth_params(n_keys, n_ops, n_dc, t, seed=0x5EED + 2):
    p = abi.am_synth_params()
    p.seed, p.n_keys, p.ops_per_key, p.n_dc, p.type, p.key_base, p.max_lag = seed, n_keys, n_ops, n_dc, t, 0, 8
    return p


def _host_log_from_synth(p, k0, nk):
    import ctypes
    n_ops = ctypes.c_uint64()
    abi.check(abi.lib().am_synth_host_sizes(ctypes.byref(p), k0, nk, ctypes.byref(n_ops), None), "sizes")
    n = n_ops.value
    log = HostLog.__new__(HostLog)
    log.n_dc, log.n_keys, log.n_ops, log.n_var, log.has_var = p.n_dc, nk, n, 0, False
    log.key_off = np.zeros(nk + 1, np.uint64)
    log.key_type = np.zeros(nk, np.uint8)
    log.key_flags = None
    log.key_id_base = None
    log.op_meta = np.zeros(n, np.uint8)
    log.commit_time = np.zeros(n, np.uint64)
    log.snap_vc = np.zeros((p.n_dc, n), np.uint64)
    log.snap_pres = None
    log.op_txid = log.op_id = None
    log.p0 = np.zeros(n, np.uint64)
    log.p1 = np.zeros(n, np.uint64)
    log.var_off = log.var_data = None
    s = log.as_struct()
    abi.check(abi.lib().am_synth_host(ctypes.byref(p), k0, nk, ctypes.byref(s)), "am_synth_host")
    return log


@pytest.mark.parametrize("t,n_dc,n_ops", [(abi.AM_LWW, 3, 256), (abi.AM_PN, 1, 64), (abi.AM_LWW, 8, 100)])
def test_gpu_synth_device_vs_oracle(mat, t, n_dc, n_ops):
    """Device-generated log (the bench's input) read at two snapshot quantiles, fresh
    and from the cached q=0.5 result; sampled keys checked against the oracle on the
    host-regenerated log."""
    from antidote_amd.devbatch import DeviceReads, materialize
    import ctypes
    n_keys = 20000
    p = _synth_params(n_keys, n_ops, n_dc, t)
    st = mat.synth_store(p)
    dlog = st.device_log()
    rng = np.random.default_rng(1)
    sample = np.sort(rng.choice(n_keys, 300, replace=False))
    hlog_full = _host_log_from_synth(p, 0, n_keys)
    prev = None
    for q in (0.5, 0.75):
        clock = (ctypes.c_uint64 * n_dc)()
        abi.lib().am_synth_read_clock(ctypes.byref(p), q, clock)
        clock = list(clock)
        dr = DeviceReads(n_keys, n_dc, t, clock)
        if prev is not None:
            dr.set_base_from(prev)
        torch.cuda.synchronize()
        materialize(mat, dlog, dr)
        mat.sync()
        got = dr.host()
        # oracle on the sampled keys
        reads = []
        for k in sample:
            base_clock = base_last = base_val = None
            if prev is not None:
                ph = prev_host
                if not ph["last_ct_ignore"][k]:
                    base_clock = {d: int(ph["last_ct"][d, k]) for d in range(n_dc) if (int(ph["last_ct_pres"][k]) >> d) & 1}
                base_last = int(ph["new_last_op"][k])
                base_val = int(ph["v0"][k]) if t == abi.AM_PN else (int(np.int64(ph["v0"][k]).view(np.uint64)),
                                                                      int(ph["v1"][k]), bool(ph["vflag"][k]))
            reads.append(Read(int(k), t, {d: clock[d] for d in range(n_dc)}, None, base_clock, base_last or 0,
                              base_val))
        ref = amo.materialize(hlog_full, HostBatch(n_dc, reads))
        for j, k in enumerate(sample):
            r = ref.result(j)
            assert r[0] == "ok"
            assert got["status"][k] == 0
            assert got["new_last_op"][k] == r[2]
            assert got["count"][k] == r[5]
            assert bool(got["is_new_ss"][k]) == r[4]
            ct = None if got["last_ct_ignore"][k] else {d: int(got["last_ct"][d, k]) for d in range(n_dc)
                                                         if (int(got["last_ct_pres"][k]) >> d) & 1}
            assert ct == r[3]
            if t == abi.AM_PN:
                assert got["v0"][k] == r[1]
            else:
                assert (int(np.int64(got["v0"][k]).view(np.uint64)), int(got["v1"][k]), bool(got["vflag"][k])) == r[1]
        # size-independent properties over ALL keys
        assert (got["status"] == 0).all()
        assert (got["count"] <= n_ops).all()
        if q == 0.75 and prev is not None:
            assert (got["count"] >= 0).all()
        prev, prev_host = dr, got
    st.close()


def test_gpu_gst(mat):
    """am_gst_local_min + am_gst_finalize (+ RCCL all-reduce at nranks=1) vs the oracle."""
    import ctypes
    rng = np.random.default_rng(5)
    for trial in range(20):
        nd, npart = int(rng.integers(1, 6)), int(rng.integers(1, 9))
        vc = rng.integers(0, 1000, size=(npart, nd)).astype(np.uint64)
        pres = rng.integers(0, 1 << nd, size=npart).astype(np.uint32)
        undef = (rng.random(npart) < 0.1).astype(np.uint8)
        out = np.zeros(nd, np.uint64)
        op = np.zeros(1, np.uint32)
        amo.lib().amo_gst_min(nd, npart, vc.ctypes.data, pres.ctypes.data, undef.ctypes.data, out.ctypes.data,
                              op.ctypes.data)
        d_vc = torch.from_numpy(vc.view(np.int64)).cuda()
        d_pres = torch.from_numpy(pres.view(np.int32)).cuda()
        d_undef = torch.from_numpy(undef).cuda()
        lanes = torch.zeros(nd + 1, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        abi.check(mat.L.am_gst_local_min(mat.ctx, nd, npart, d_vc.data_ptr(), d_pres.data_ptr(), d_undef.data_ptr(),
                                         lanes.data_ptr()), "local_min")
        mat.sync()
        ln = lanes.cpu().numpy().view(np.uint64)
        for d in range(nd):
            if (int(op[0]) >> d) & 1:
                assert ln[d] == out[d]
            else:
                assert ln[d] == np.uint64(0xFFFFFFFFFFFFFFFF)
        # finalize against a previous stable snapshot
        last = rng.integers(0, 800, size=nd).astype(np.uint64)
        lastp = np.array([rng.integers(0, 1 << nd)], np.uint32)
        h_last, h_lastp = last.copy(), lastp.copy()
        changed_ref = amo.lib().amo_update_stable(nd, h_last.ctypes.data, h_lastp.ctypes.data, out.ctypes.data,
                                                  int(op[0]))
        d_last = torch.from_numpy(last.view(np.int64)).cuda()
        d_lastp = torch.from_numpy(lastp.view(np.int32)).cuda()
        o_vc = torch.zeros(nd, dtype=torch.int64, device="cuda")
        o_p = torch.zeros(1, dtype=torch.int32, device="cuda")
        ch = torch.zeros(1, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        abi.check(mat.L.am_gst_finalize(mat.ctx, nd, lanes.data_ptr(), d_last.data_ptr(), d_lastp.data_ptr(), 0,
                                        o_vc.data_ptr(), o_p.data_ptr(), ch.data_ptr()), "finalize")
        mat.sync()
        assert int(ch.item()) == changed_ref
        assert int(d_lastp.item()) & 0xFFFFFFFF == int(h_lastp[0])
        gv = d_last.cpu().numpy().view(np.uint64)
        for d in range(nd):
            if (int(h_lastp[0]) >> d) & 1:
                assert gv[d] == h_last[d]


def test_gpu_rccl_single_rank(mat):
    import ctypes
    uid = (ctypes.c_char * 128)()
    abi.check(mat.L.am_comm_unique_id(uid), "uid")
    comm = ctypes.c_void_p()
    abi.check(mat.L.am_comm_init(mat.ctx, 0, 1, uid, ctypes.byref(comm)), "comm_init")
    lanes = torch.tensor([5, 7, 1], dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    abi.check(mat.L.am_gst_allreduce(comm, lanes.data_ptr(), 2), "allreduce")
    mat.sync()
    assert lanes.cpu().tolist() == [5, 7, 1]
    mat.L.am_comm_destroy(comm)


def test_gpu_set_lds_overflow_goes_big(mat):
    """A read whose births exceed one workgroup's LDS lists (1100 concurrent MV values)
    is handed to the big-read tier (am_big.hip) and still matches the oracle."""
    ops = [Op(abi.AM_MVREG, 0, 10 + i, {0: 1}, ("assign", i, 1000 + i, [])) for i in range(1100)]
    log = HostLog(1, [ops])
    got = _batch_compare(log, [Read(0, abi.AM_MVREG, {0: 10**6})], mat, 1, cap=4096)
    assert got.result(0)[0] == "ok" and len(got.result(0)[1]) == 1100


def _big_key_ops(rng, t, n_dc, n_ops, partial, txids, bad_rate, concurrent):
    ops = randlog.rand_key_ops(rng, t, n_dc, n_ops, partial=partial, txids=txids, bad_rate=bad_rate,
                               t0=rng.randint(0, 50))
    if concurrent and t == abi.AM_MVREG:  # many survivors: assigns that override nothing
        for op in ops:
            if not op.bad and op.effect[0] == "assign" and rng.random() < 0.7:
                op.effect = ("assign", op.effect[1], op.effect[2], [])
    return ops


@pytest.mark.parametrize("t", SET_TYPES + (abi.AM_BCOUNTER,))
@pytest.mark.parametrize("seed", range(3))
def test_gpu_big_reads(mat, t, seed):
    """Set-CRDT reads beyond the LDS tier (thousands of ops: chunked over workgroups with
    local resolution + global hash), mixed with short reads of the same batch; partial
    clocks, TxIds, cached bases, invalid effects, > 2048 survivors (global-memory sort)."""
    rng = random.Random(7000 + seed * 13 + t)
    n_dc = [2, 3, 8][seed]
    partial, txids = seed == 1, seed == 2
    keys, reads = [], []
    lens = [0, 5, 300, 1500, 4100, 9000, 20000]
    for k in range(12):
        n_ops = lens[k % len(lens)]
        keys.append(_big_key_ops(rng, t, n_dc, n_ops, partial, txids, 0.0005 if seed == 1 else 0.0,
                                 concurrent=k % 3 == 0))
        hi = keys[-1][-1].commit_time if keys[-1] else 50
        q = rng.choice([0.3, 0.8, 1.0])
        clock = randlog.rand_clock(rng, n_dc, int(hi * q), int(hi * q) + 6, partial=partial)
        reads.append(Read(k, t, clock, rng.choice([None, 1, 3]) if txids else None))
    log = HostLog(n_dc, keys, key_types=[t] * len(keys), partial=partial or None)
    first = _batch_compare(log, reads, mat, n_dc, cap=16384)
    reads2 = []
    for i, r in enumerate(reads):
        res = first.result(i)
        if res[0] != "ok":
            continue
        clock2 = {d: v + rng.randint(0, 20000) for d, v in r.clock.items()}
        reads2.append(Read(r.key, t, clock2, None, res[3], res[2], res[1]))
    _batch_compare(log, reads2, mat, n_dc, cap=16384)


@pytest.mark.parametrize("seed", range(3))
def test_gpu_mixed_type_batches(mat, seed):
    """One batch mixing all five CRDT types (the planner partitions it on the device),
    plus unknown keys / types and keys whose log holds another type."""
    rng = random.Random(9100 + seed)
    n_dc = [1, 3, 6][seed]
    keys, types = [], []
    for k in range(150):
        t = randlog.TYPES[k % 5]
        n_ops = rng.choice([0, 1, 7, 16, 64, 300, 5000 if k % 37 == 0 else 90])
        keys.append(randlog.rand_key_ops(rng, t, n_dc, n_ops, partial=seed == 2, txids=seed == 1))
        types.append(t)
    log = HostLog(n_dc, keys, key_types=types, partial=(seed == 2) or None)
    reads = []
    for i in rng.sample(range(450), 450):
        k = i % 150
        t = types[k] if i < 420 else randlog.TYPES[(k + 1) % 5]  # tail: wrong type -> corrupted
        hi = keys[k][-1].commit_time if keys[k] else 50
        reads.append(Read(k, t, randlog.rand_clock(rng, n_dc, hi // 2, hi + 5, partial=seed == 2),
                          rng.choice([None, 2]) if seed == 1 else None))
    first = _batch_compare(log, reads, mat, n_dc, cap=8192)
    assert any(first.result(i)[0] == "error" for i in range(len(reads)))
    reads2 = []
    for i, r in enumerate(reads):
        res = first.result(i)
        if res[0] == "ok":
            reads2.append(Read(r.key, r.type, {d: v + 40 for d, v in r.clock.items()}, None, res[3], res[2], res[1]))
    _batch_compare(log, reads2, mat, n_dc, cap=8192)


def test_gpu_reference_system_shapes(mat):
    """Value shapes the reference's system tests assert (test/singledc/clocksi_SUITE.erl:160-205):
    AW-set add a, add b, remove a -> [b]; MV register a -> b -> c -> [c]."""
    a, b = 97, 98
    aw = [Op(abi.AM_AWSET, 0, 11, {0: 10}, [(a, [1], [])]),
          Op(abi.AM_AWSET, 0, 12, {0: 11}, [(b, [2], [])]),
          Op(abi.AM_AWSET, 0, 13, {0: 12}, [(a, [], [1])])]
    mv = [Op(abi.AM_MVREG, 0, 11, {0: 10}, ("assign", 1, 7, [])),
          Op(abi.AM_MVREG, 0, 12, {0: 11}, ("assign", 2, 8, [7])),
          Op(abi.AM_MVREG, 0, 13, {0: 12}, ("assign", 3, 9, [8]))]
    for t, ops, exp in ((abi.AM_AWSET, aw, [(b, 2)]), (abi.AM_MVREG, mv, [(3, 9)])):
        log = HostLog(1, [ops])
        got = _batch_compare(log, [Read(0, t, {0: 20})], mat, 1)
        assert got.result(0)[1] == exp


@pytest.mark.parametrize("t", [abi.AM_PN, abi.AM_LWW])
def test_gpu_packed_view_escapes(mat, t):
    """Ops whose snapshot entries lie > 2^31 us from the commit time, or whose commit time
    is >= 2^55, do not fit the packed streaming view: they are flagged and read from the
    full columns.  Mix fitting and escaping ops in one log, read at several clocks."""
    rng = random.Random(77 + t)
    big = 2**40
    keys, reads = [], []
    for k in range(40):
        ops = []
        ct = 10**6
        for i in range(rng.choice([5, 100, 300])):
            ct += rng.randint(1, 3)
            mode = rng.random()
            if mode < 0.1:
                c, snap = ct + big, {0: ct - 5, 1: ct + big - 7, 2: 3}             # far behind
            elif mode < 0.15:
                c, snap = 2**55 + ct, {0: 2**55 + ct - 1, 1: 2**55, 2: 2**55 + 1}  # >= 2^55
            elif mode < 0.2:
                c, snap = ct, {0: ct + 2**33, 1: ct - 1, 2: ct - 2}                  # skewed ahead
            else:
                c, snap = ct, {d: ct - rng.randint(1, 50) for d in range(3)}
            dc = rng.randrange(3)
            eff = rng.randint(-9, 9) if t == abi.AM_PN else (rng.randint(1, 10**6), rng.randint(0, 9))
            ops.append(Op(t, dc, c, snap, eff))
        keys.append(ops)
        top = max(op.commit_time for op in ops)
        clock = {d: rng.choice([ct, ct + big, top, 2**55 + ct + 10, 2**62]) for d in range(3)}
        reads.append(Read(k, t, clock))
    log = HostLog(3, keys, key_types=[t] * len(keys))
    _batch_compare(log, reads, mat, 3)


@pytest.mark.parametrize("t", GPU_TYPES)
@pytest.mark.parametrize("n_dc", [1, 3, 8])
def test_gpu_packed_view_time_base(mat, t, n_dc):
    """The packed view stores each op's commit vector as u32 offsets from a per-key time base
    (include/antidote_mat.h key_tbase / pk_vc).  With wall-clock microsecond timestamps the
    base is non-zero; ops with an entry below the base or 2^32 above it (a snapshot entry
    far behind, a late commit, a key whose log spans hours), and a first op with a stale
    entry (left out of the base), must read like the rest.  Read clocks below the base,
    inside the window and far above it; then incremental reads against the cached base clock
    (belongs_to_snapshot_op on the packed view)."""
    rng = random.Random(4242 + 17 * t + n_dc)
    T0 = 1_700_000_000_000_000
    keys, reads = [], []
    for k in range(48):
        n_ops = rng.choice([1, 5, 40, 130, 300]) if t in SET_TYPES else rng.choice([1, 5, 40, 130, 300, 900])
        ops = randlog.rand_key_ops(rng, t, n_dc, n_ops, t0=T0 + rng.randint(0, 10**6))
        mode = k % 6
        for i, op in enumerate(ops):
            x = rng.random()
            if mode == 1 and x < 0.1:    # a snapshot entry far behind
                op.snap[rng.randrange(n_dc)] = op.commit_time - 2**32 - rng.randint(0, 99)
            elif mode == 2 and x < 0.1:  # a late commit (clock jump)
                op.commit_time += 2**33
            elif mode == 3 and i >= n_ops // 2:  # the log spans more than 2^32 us
                op.commit_time += 2**32 + 5
                op.snap = {d: v + 2**32 for d, v in op.snap.items()}
            elif mode == 4 and i == 0:   # stale entry in the first op
                op.snap[rng.randrange(n_dc)] = 7
        keys.append(ops)
        lo, hi = min(op.commit_time for op in ops), max(op.commit_time for op in ops)
        clock = {d: rng.choice([lo - 2**31, lo - 5, (lo + hi) // 2, hi, hi + 2**32, 2**63 + 1])
                 for d in range(n_dc)}
        reads.append(Read(k, t, clock))
    log = HostLog(n_dc, keys, key_types=[t] * len(keys))
    first = _batch_compare(log, reads, mat, n_dc)
    reads2 = []
    for i, r in enumerate(reads):
        res = first.result(i)
        if res[0] == "ok":
            clock2 = {d: v + rng.choice([0, 3, 2**31]) for d, v in r.clock.items()}
            reads2.append(Read(r.key, t, clock2, None, res[3], res[2], res[1]))
    _batch_compare(log, reads2, mat, n_dc)


def _seq_ops(t, effects, n_dc=2):
    return [Op(t, i % n_dc, 10 + 2 * i, {d: 10 + 2 * i - 1 for d in range(n_dc)}, eff) for i, eff in enumerate(effects)]


def test_gpu_group_tier_guards(mat):
    """The token-group tier (am_group.hip) serves keys whose log the group builder could
    number; the others go to the var_data tiers.  Every case must match the oracle.
    Logs of 60 .. 2100 ops:
      0  AW: one token under two elems (two kill keys (elem, tok): two groups)
      1  AW: 600 live elems (600 survivors)
      2  MV: one token with two values (outside the closed form: ungrouped, LDS-sort tier)
      3  MV: 1500 concurrent values (1500 groups)
      4  AW / 5 MV: the sentinel 2^64-1 as a token / value
      6  AW: plain 300-op log, 7  MV: plain 2000-op chain
      8  AW: 2100 ops, ~4200 births/kills (beyond the group view: the LDS-sort tier)"""
    M = (1 << 64) - 1
    aw, mv = abi.AM_AWSET, abi.AM_MVREG
    keys, types = [], []

    def add(t, effs):
        keys.append(_seq_ops(t, effs))
        types.append(t)

    add(aw, [[(i % 7, [900 + (i % 40)], [])] for i in range(80)])
    add(aw, [[(i, [1000 + i], [])] for i in range(600)])
    add(mv, [("assign", i % 3, 77 if i % 10 == 0 else 500 + i, []) for i in range(90)])
    add(mv, [("assign", i, 3000 + i, []) for i in range(1500)])
    add(aw, [[(1, [M if i == 30 else 5000 + i], [])] for i in range(70)])
    add(mv, [("assign", M if i == 40 else i, 6000 + i, [6000 + i - 1] if i else []) for i in range(70)])
    effs, live = [], {}
    for i in range(300):
        e = i % 9
        effs.append([(e, [7000 + i], live.get(e, []))])
        live[e] = [7000 + i]
    add(aw, effs)
    add(mv, [("assign", i % 5, 9000 + i, [9000 + i - 1] if i else []) for i in range(2000)])
    add(aw, [[(i % 11, [20000 + i], [20000 + i - 11] if i >= 11 else [])] for i in range(2100)])
    log = HostLog(2, keys, key_types=types)
    reads = []
    for k, ops in enumerate(keys):
        hi = ops[-1].commit_time
        for q in (0.5, 1.0):
            c = int(10 + (hi - 10) * q)
            reads.append(Read(k, types[k], {0: c, 1: c}))
    got = _batch_compare(log, reads, mat, 2, cap=4096)  # mixed batch: the planner splits it
    assert got.result(3)[0] == "ok"  # key 1 at q=1.0: 600 survivors
    for t in (aw, mv):  # single-type batches (type_hint path)
        _batch_compare(log, [r for r in reads if r.type == t], mat, 2, cap=4096)


def test_gpu_group_tier_mixed_batch(mat):
    """The group tier inside a mixed batch (planner selection + row-kernel hand-off list),
    then cached bases (base pairs: the LDS-sort tier) on the second read."""
    rng = random.Random(4242)
    keys, types = [], []
    for k in range(60):
        t = [abi.AM_AWSET, abi.AM_MVREG, abi.AM_PN][k % 3]
        keys.append(randlog.rand_key_ops(rng, t, 3, rng.choice([10, 70, 200, 900, 1900])))
        types.append(t)
    log = HostLog(3, keys, key_types=types)
    reads = []
    for k, ops in enumerate(keys):
        hi = ops[-1].commit_time
        reads.append(Read(k, types[k], randlog.rand_clock(rng, 3, int(hi * 0.6), int(hi * 0.6) + 8)))
    first = _batch_compare(log, reads, mat, 3, cap=4096)
    reads2 = []
    for i, r in enumerate(reads):
        res = first.result(i)
        if res[0] == "ok":
            clock2 = {d: v + rng.randint(0, 3000) for d, v in r.clock.items()}
            reads2.append(Read(r.key, r.type, clock2, None, res[3], res[2], res[1]))
    _batch_compare(log, reads2, mat, 3, cap=4096)
