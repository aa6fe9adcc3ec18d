"""The chunked token-group view of hot MV-register keys (am_grpbig.hip: device-wide segmented
sorts build the groups of keys with more than AM_GRP_MAX_REC ops) and the big-read tier's
grouped mode over it (am_big.hip: per-chunk record streaming into born / killed group
bitmaps), against the oracle.  Bar: bit-exact on every output column."""
import random

import numpy as np
import pytest

from antidote_amd import abi
from antidote_amd.oplog import HostBatch, HostLog, Op, Read
from oracle import amo
from tests import randlog

pytestmark = pytest.mark.gpu

NGRP_BIG = 0x80000000
NGRP_NONE = 0xFFFFFFFF


@pytest.fixture(scope="module")
def mat():
    from antidote_amd.materializer import Materializer
    m = Materializer(0)
    yield m
    m.close()


def _ngrp(mat, st, n_keys):
    L = st.device_log()
    out = np.zeros(max(n_keys, 1), np.uint32)
    abi.check(mat.L.am_memcpy_d2h(mat.ctx, out.ctypes.data, L.key_ngrp, out.nbytes), "am_memcpy_d2h")
    return out[:n_keys]


def _compare(mat, log, reads, cap):
    st = mat.store(log)
    try:
        ng = _ngrp(mat, st, log.n_keys)
        caps = [cap] * len(reads)
        got = mat.read_batch(st, reads, caps)
    finally:
        st.close()
    ref = amo.materialize(log, HostBatch(log.n_dc, reads, caps))
    for i in range(len(reads)):
        a, b = got.result(i), ref.result(i)
        assert a == b, (i, reads[i].key, a[:1], b[:1])
    return got, ng


def _chain(n_dc, n_ops, t0=10, vals=1000):
    """An MV override chain (the C5 synthetic shape): op i assigns (v_i, tok i) over tok i-1."""
    ops, ct = [], t0
    for i in range(n_ops):
        ct += 3
        dc = i % n_dc
        snap = {d: ct - 1 - ((i + d) % 5) for d in range(n_dc)}
        ops.append(Op(type=abi.AM_MVREG, commit_dc=dc, commit_time=ct, snap=snap,
                      effect=("assign", (i * 7919) % vals, 10_000 + i, [10_000 + i - 1] if i else [])))
    return ops


@pytest.mark.parametrize("n_dc", [3, 16])
def test_gpu_chunked_view_chains(mat, n_dc):
    """Override chains of 1025 .. 70000 ops (beyond the LDS builder, one above the old 2^16-op
    limit) read at several snapshot quantiles; short keys in the same batch."""
    lens = [0, 40, 1024, 1025, 2049, 5000, 70000, 9001]
    keys = [_chain(n_dc, n) for n in lens]
    log = HostLog(n_dc, keys, key_types=[abi.AM_MVREG] * len(keys))
    reads = []
    for k, ops in enumerate(keys):
        hi = ops[-1].commit_time if ops else 50
        for q in (0.0, 0.37, 0.999, 1.2):
            reads.append(Read(k, abi.AM_MVREG, {d: int(hi * q) + d for d in range(n_dc)}))
    got, ng = _compare(mat, log, reads, cap=64)
    for k, n in enumerate(lens):
        if n > 1024:  # one group per token
            assert int(ng[k]) == (NGRP_BIG | n), (k, hex(int(ng[k])))
        else:         # the LDS builder's (1024 ops hold 2047 records)
            assert int(ng[k]) == NGRP_NONE or not int(ng[k]) & NGRP_BIG, (k, hex(int(ng[k])))


@pytest.mark.parametrize("seed", range(3))
def test_gpu_chunked_view_random(mat, seed):
    """Random MV logs (resets, partial overrides -> many survivors, equal values so the
    (value, token) order has ties) with partial clocks, TxIds, invalid effects; then the
    same reads from the first results as cached bases (those go to the var_data path)."""
    rng = random.Random(9100 + seed)
    n_dc = [2, 5, 8][seed]
    partial, txids = seed == 1, seed == 2
    keys, reads = [], []
    for k in range(10):
        n_ops = [2100, 3000, 6000, 12000, 100, 0][k % 6]
        ops = randlog.rand_key_ops(rng, abi.AM_MVREG, n_dc, n_ops, partial=partial, txids=txids,
                                   bad_rate=0.0005 if seed == 1 else 0.0, t0=rng.randint(0, 50))
        keys.append(ops)
        hi = ops[-1].commit_time if ops else 50
        for q in (0.2, 0.9, 1.0):
            clock = randlog.rand_clock(rng, n_dc, int(hi * q), int(hi * q) + 6, partial=partial)
            reads.append(Read(k, abi.AM_MVREG, clock, rng.choice([None, 1, 3]) if txids else None))
    log = HostLog(n_dc, keys, key_types=[abi.AM_MVREG] * len(keys), partial=partial or None)
    first, ng = _compare(mat, log, reads, cap=8192)
    assert any(int(x) != NGRP_NONE and int(x) & NGRP_BIG for x in ng)
    reads2 = []
    for i, r in enumerate(reads):
        res = first.result(i)
        if res[0] != "ok":
            continue
        clock2 = {d: v + rng.randint(0, 3000) for d, v in r.clock.items()}
        reads2.append(Read(r.key, abi.AM_MVREG, clock2, None, res[3], res[2], res[1]))
    _compare(mat, log, reads2, cap=8192)


def test_gpu_chunked_view_token_born_twice(mat):
    """A hot key whose log assigns one token twice is outside the closed form: it stays
    ungrouped (AM_NGRP_NONE) and reads through var_data."""
    ops = _chain(3, 3000)
    e = ops[2500].effect
    ops[2500].effect = (e[0], e[1], 10_000 + 100, e[3])  # tok 100 again
    log = HostLog(3, [ops], key_types=[abi.AM_MVREG])
    hi = ops[-1].commit_time
    _, ng = _compare(mat, log, [Read(0, abi.AM_MVREG, {d: hi for d in range(3)})], cap=64)
    assert int(ng[0]) == NGRP_NONE


def test_gpu_stale_type_cache_log_without_groups(mat):
    """The per-log type mask is cached on the context by the key_type pointer (am_plan.hip
    log_types) and may be stale: a log that shares key_type with a big-MV store but has no
    token-group view (key_ngrp / rec_g / gmask absent) must still read correctly -- the early
    big-MV class and the lane tier's metadata loads guard on the log itself."""
    import ctypes

    import torch

    from antidote_amd.devbatch import DeviceReads, materialize
    rng = random.Random(11)
    n_dc = 3
    keys = [_chain(n_dc, 2000)] + [randlog.rand_key_ops(rng, abi.AM_PN, n_dc, rng.choice([0, 5, 16])) for _ in range(40)]
    keys += [_chain(n_dc, 7)]
    types = [abi.AM_MVREG] + [abi.AM_PN] * 40 + [abi.AM_MVREG]
    log = HostLog(n_dc, keys, key_types=types)
    st = mat.store(log)
    try:
        full = st.device_log()
        bare = abi.am_op_log()
        ctypes.pointer(bare)[0] = full
        for f in ("key_ngrp", "rec_key_off", "rec_key_end", "rec_g", "grp", "gmask", "zone_vc", "zone_gsum"):
            setattr(bare, f, None)
        bare.n_rec = 0
        clock = [10 ** 6] * n_dc
        tt = torch.tensor(types, dtype=torch.uint8, device="cuda")
        for L in (full, bare, full, bare):  # the mask is cached from the first (full) log
            dr = DeviceReads(len(keys), n_dc, 0, clock, set_cap=64, types=tt)
            materialize(mat, L, dr)
            mat.sync()
            reads = [Read(k, types[k], {d: clock[d] for d in range(n_dc)}) for k in range(len(keys))]
            ref = amo.materialize(log, HostBatch(n_dc, reads, [64] * len(keys)))
            h = dr.host()
            vals = dr.values(range(len(keys)))
            for i in range(len(keys)):
                ct = None if h["last_ct_ignore"][i] else {d: int(h["last_ct"][d, i]) for d in range(n_dc)
                                                          if (int(h["last_ct_pres"][i]) >> d) & 1}
                got = ("ok", vals[i], int(h["new_last_op"][i]), ct, bool(h["is_new_ss"][i]), int(h["count"][i]),
                       int(h["flags"][i])) if h["status"][i] == 0 else ("error", int(h["status"][i]))
                assert got == ref.result(i), (i, got, ref.result(i))
    finally:
        st.close()
