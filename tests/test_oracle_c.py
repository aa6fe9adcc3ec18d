"""Pin the C oracle (oracle/am_oracle.c, the checker used at scale and the CPU baseline)
to the Python restatement, which is itself pinned by the reference's EUnit KATs."""
import random

import numpy as np
import pytest

from antidote_amd import abi
from antidote_amd.oplog import HostBatch, HostLog, Op, Read
from oracle import amo
from tests import randlog
from tests.kat_util import load

KAT = load("kat_materialize.json")


def _dcmap(kat):
    dcs = set()
    for _, p in kat["ops"]:
        dcs.add(p["commit"][0])
        dcs |= {d for d, _ in p["ss"]}
    for c in kat["cases"]:
        dcs |= {d for d, _ in c["read"]}
    return {d: i for i, d in enumerate(sorted(dcs))}


def kat_ops(kat, m):
    ops = []
    for i, p in reversed(kat["ops"]):     # oldest first
        ops.append(Op(type=kat["type"], commit_dc=m[p["commit"][0]], commit_time=p["commit"][1],
                      snap={m[d]: t for d, t in p["ss"]}, effect=p["param"], txid=p["txid"], op_id=i))
    return ops


def run_kat_cases(kat, run_one):
    """Drive a KAT's cases through run_one(read) -> ABI result tuple; returns the results."""
    m = _dcmap(kat)
    outs = []
    for case in kat["cases"]:
        if "base_from" in case:
            prev = outs[case["base_from"]]
            read = Read(0, kat["type"], {m[d]: t for d, t in case["read"]}, None, prev[3], prev[2], prev[1])
        else:
            b = case["base"]
            read = Read(0, kat["type"], {m[d]: t for d, t in case["read"]}, None,
                        None if b["ct"] is None else {m[d]: t for d, t in b["ct"]}, b["last_op"], b["value"])
        r = run_one(read)
        assert r[0] == "ok", r
        outs.append(r)
        exp = case["expect"]
        assert r[1] == exp["value"]
        if "new_last_op" in exp:
            assert r[2] == exp["new_last_op"]
        if "last_op_ct" in exp:
            assert r[3] == (None if exp["last_op_ct"] is None else {m[d]: t for d, t in exp["last_op_ct"]})
        if "is_new_ss" in exp:
            assert r[4] == exp["is_new_ss"]
        if "count" in exp:
            assert r[5] == exp["count"]
    return outs


def oracle_one(ops, n_dc, read, key_type=None):
    log = HostLog(n_dc, [ops], key_types=[key_type if key_type is not None else read.type])
    hb = HostBatch(n_dc, [read])
    amo.materialize(log, hb)
    return hb.result(0)


@pytest.mark.parametrize("kat", KAT["materialize"], ids=lambda k: k["name"])
def test_c_oracle_kat(kat):
    m = _dcmap(kat)
    ops = kat_ops(kat, m)
    run_kat_cases(kat, lambda read: oracle_one(ops, max(len(m), 1), read))


def _compare(a, b):
    assert a[0] == b[0], (a, b)
    if a[0] == "error":
        assert a[1] == b[1], (a, b)
        return
    assert a[1:] == b[1:], (a, b)


@pytest.mark.parametrize("t", randlog.TYPES)
@pytest.mark.parametrize("seed", range(6))
def test_c_oracle_vs_python_random(t, seed):
    rng = random.Random(seed * 101 + t)
    n_dc = rng.choice([1, 2, 3, 5])
    partial = seed % 2 == 1
    for trial in range(12):
        ops = randlog.rand_key_ops(rng, t, n_dc, rng.randint(0, 40), partial=partial, txids=seed % 3 == 0,
                                   bad_rate=0.03 if seed == 4 else 0.0)
        hi = ops[-1].commit_time if ops else 20
        clock = randlog.rand_clock(rng, n_dc, 0, hi + 5, partial=partial)
        read = Read(0, t, clock, rng.choice([None, 1, 2]) if seed % 3 == 0 else None)
        ref = randlog.ref_materialize(t, ops, read)
        got = oracle_one(ops, n_dc, read)
        _compare(got, ref)
        if got[0] == "ok":
            # incremental read from the cached result (exercises belongs_to_snapshot_op)
            clock2 = {d: v + rng.randint(0, 20) for d, v in clock.items()}
            read2 = Read(0, t, clock2, None, got[3], got[2], got[1])
            _compare(oracle_one(ops, n_dc, read2), randlog.ref_materialize(t, ops, read2))


def test_c_oracle_corrupted_and_empty():
    ops = [Op(abi.AM_PN, 0, 5, {0: 1}, 3)]
    r = oracle_one(ops, 1, Read(0, abi.AM_LWW, {0: 10}))
    assert r == ("error", abi.AM_ERR_CORRUPTED_OPS_CACHE)
    r = oracle_one([], 1, Read(0, abi.AM_LWW, {0: 10}))
    assert r == ("ok", (0, 0, True), 0, None, False, 0, 0)


def test_c_oracle_pn_overflow():
    ops = [Op(abi.AM_PN, 0, 5 + i, {0: 1}, 2**62) for i in range(3)]
    assert oracle_one(ops, 1, Read(0, abi.AM_PN, {0: 100})) == ("error", abi.AM_ERR_OVERFLOW)
    ops2 = [Op(abi.AM_PN, 0, 5 + i, {0: 1}, v) for i, v in enumerate([2**62, 2**62, -2**62, -2**62 + 7])]
    assert oracle_one(ops2, 1, Read(0, abi.AM_PN, {0: 100}))[1] == 7   # intermediate overflow is fine


def test_c_oracle_gst_kats():
    from tests.kat_util import load as ld
    from oracle import ref_materializer as R
    import ctypes
    vn = ld("kat_vnode.json")
    for case in vn["gst"]:
        table = {p: {d: t for d, t in c} for p, c in case["table"].items()}
        local = R.local_partition_dicts(case["partitions"], table, case["check_nodes"])
        dcs = sorted({d for c in table.values() for d in c})
        m = {d: i for i, d in enumerate(dcs)}
        nd = max(len(dcs), 1)
        parts = list(local.items())
        vc = np.zeros((max(len(parts), 1), nd), np.uint64)
        pres = np.zeros(max(len(parts), 1), np.uint32)
        undef = np.zeros(max(len(parts), 1), np.uint8)
        for i, (_, dct) in enumerate(parts):
            if dct == R.UNDEFINED:
                undef[i] = 1
                continue
            for d, t in dct.items():
                vc[i, m[d]] = t
                pres[i] |= 1 << m[d]
        out = np.zeros(nd, np.uint64)
        op = np.zeros(1, np.uint32)
        amo.lib().amo_gst_min(nd, len(parts), vc.ctypes.data, pres.ctypes.data, undef.ctypes.data,
                              out.ctypes.data, op.ctypes.data)
        got = {d: int(out[m[d]]) for d in dcs if (int(op[0]) >> m[d]) & 1}
        assert got == {d: t for d, t in case["expect"]}, case["name"]
