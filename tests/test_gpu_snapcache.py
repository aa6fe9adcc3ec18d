"""The device snapshot cache (am_snapcache_read) against the oracle's
materializer_vnode:internal_read/7 (oracle/ref_materializer.py: get_from_snapshot_cache,
vector_orddict get_smaller / insert_bigger, materialize_snapshot, internal_store_ss,
snapshot_insert_gc; src/materializer_vnode.erl:342-509, src/vector_orddict.erl:75-140).

Bar: bit-exact read values and statuses (LogColdPath <-> AM_ERR_COLD_PATH), and the cache
contents after every batch (clocks, last_op_id, values, newest first)."""
import random

import pytest

from antidote_amd import abi
from antidote_amd.oplog import HostLog, Read
from oracle import ref_materializer as R
from tests import randlog

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mat():
    from antidote_amd.materializer import Materializer
    m = Materializer(0)
    yield m
    m.close()


def _oracle_state(keys, types):
    st = R.VnodeState()
    for k, ops in enumerate(keys):
        if not ops:
            continue
        payloads = [(i + 1, randlog.payload_term(op, key=k)) for i, op in enumerate(ops)]
        st.ops_cache[k] = R.OpsTuple(k, len(ops), max(50, len(ops)), len(ops), payloads)
    return st


def _canon_entry(t, snap):
    v = randlog.canon_state(t, snap.value)
    return snap.last_op_id, v


def _dev_value(t, v0, v1, vflag):
    if t == abi.AM_PN:
        return v0
    return (v0 & (2**64 - 1), v1, bool(vflag))


@pytest.mark.parametrize("t", [abi.AM_PN, abi.AM_LWW, abi.AM_AWSET, abi.AM_MVREG, abi.AM_BCOUNTER])
@pytest.mark.parametrize("seed", range(3))
def test_gpu_snapcache_internal_read(mat, seed, t):
    """Every type's values are cached (PN / LWW in the entry, set pairs and bounded-counter
    slots in the value pool) and serve later reads as bases."""
    rng = random.Random(3300 + seed + 17 * t)
    n_dc = [1, 3, 5][seed]
    n_keys = 40
    keys, types = [], []
    for k in range(n_keys):
        kt = t if k % 2 == 0 else (abi.AM_PN if t != abi.AM_PN else abi.AM_LWW)  # two types per batch
        keys.append(randlog.rand_key_ops(rng, kt, n_dc, rng.choice([0, 3, 12, 40, 90, 200])))
        types.append(kt)
    log = HostLog(n_dc, keys, key_types=types)
    store = mat.store(log)
    cache = mat.snapshot_cache(store, n_keys)
    st = _oracle_state(keys, types)
    hi = [ops[-1].commit_time if ops else 20 for ops in keys]
    try:
        for rnd in range(12):
            sel = rng.sample(range(n_keys), 25)
            reads = []
            for k in sel:
                q = min(1.3, 0.1 * rnd + rng.choice([0.0, 0.05, 0.2])) if rng.random() < 0.85 else rng.random() * 0.5
                c = int(10 + (hi[k] - 10) * q)
                clock = {d: c + rng.randint(0, 3) for d in range(n_dc)}
                reads.append(Read(k, types[k], clock))
            dup = Read(sel[0], types[sel[0]], dict(reads[0].clock))
            got = cache.read(reads + [dup], set_capacity=[4096] * (len(reads) + 1))
            assert got.result(len(reads)) == ("error", abi.AM_ERR_INVALID)  # second read of a key in a batch
            for i, rd in enumerate(reads):
                try:
                    ref = R.internal_read(rd.key, rd.type, dict(rd.clock), R.IGNORE, False, st)
                except R.LogColdPath:
                    ref = ("cold",)
                g = got.result(i)
                if ref[0] == "cold":
                    assert g == ("error", abi.AM_ERR_COLD_PATH), (rnd, rd, g)
                elif ref[0] == "error":
                    assert g[0] == "error", (rnd, rd, g, ref)
                else:
                    assert g[0] == "ok" and g[1] == randlog.canon_state(rd.type, ref[1]), (rnd, rd, g, ref)
            for k in sel:
                dev = cache.snapshots(k, types[k])
                if k not in st.snapshot_cache:
                    assert dev is None
                    continue
                lst, size = st.snapshot_cache[k]
                assert len(dev) == size == len(lst), (rnd, k, dev, lst)
                for (clock, snap), (dclock, dlo, dval) in zip(lst, dev):
                    assert dict(clock) == dclock, (rnd, k)
                    assert _canon_entry(types[k], snap) == (dlo, dval), (rnd, k, snap, dlo, dval)
    finally:
        cache.close()
        store.close()


def test_gpu_snapcache_refresh_and_prune(mat):
    """One hot PN key read at ever newer clocks: every read adds >= MIN_OP_STORE_SS ops, so a
    snapshot is stored each time until SNAPSHOT_THRESHOLD entries prune to SNAPSHOT_MIN; an
    old clock then finds no snapshot at or below it (the log cold path)."""
    ops = randlog.rand_key_ops(random.Random(5), abi.AM_PN, 2, 400)
    log = HostLog(2, [ops], key_types=[abi.AM_PN])
    store = mat.store(log)
    cache = mat.snapshot_cache(store, 1)
    st = _oracle_state([ops], [abi.AM_PN])
    try:
        sizes = []
        for j in range(1, 14):
            c = ops[min(len(ops) - 1, 25 * j)].commit_time + 12
            rd = Read(0, abi.AM_PN, {0: c, 1: c})
            g = cache.read([rd]).result(0)
            ref = R.internal_read(0, abi.AM_PN, dict(rd.clock), R.IGNORE, False, st)
            assert g[0] == "ok" and g[1] == ref[1]
            dev = cache.entries(0)
            sizes.append(len(dev))
            assert len(dev) == st.snapshot_cache[0][1]
        assert max(sizes) >= 5
        rd = Read(0, abi.AM_PN, {0: ops[3].commit_time, 1: ops[3].commit_time})
        g = cache.read([rd]).result(0)
        try:
            ref = R.internal_read(0, abi.AM_PN, dict(rd.clock), R.IGNORE, False, st)
            assert g[0] == "ok" and g[1] == ref[1]
        except R.LogColdPath:  # the pruned dict holds no snapshot that old
            assert g == ("error", abi.AM_ERR_COLD_PATH)
    finally:
        cache.close()
        store.close()
