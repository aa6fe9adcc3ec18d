"""Op-cache ingestion + GC on the device (am_store_update, am_snapcache_gc_threshold) against
the oracle's restatement of materializer_vnode:prune_ops/2 + check_filter/7, op_insert_gc/3
and snapshot_insert_gc/4's threshold (oracle/ref_materializer.py; src/materializer_vnode.erl:
515-647, src/materializer.erl:102-106).

Bar: bit-exact -- the surviving op ids, in order, every column of every surviving / appended
op, the AM_GC_* flags, and (end to end) snapshot-cache reads through the rebuilt log."""
import random

import numpy as np
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


def _tuple(k, ops, ids=None, counter=None):
    ids = ids or list(range(1, len(ops) + 1))
    payloads = [(i, randlog.payload_term(op, key=k)) for i, op in zip(ids, ops)]
    return R.OpsTuple(k, len(ops), max(50, len(ops) + 6), counter if counter is not None else (ids[-1] if ids else 0),
                      payloads)


def _op_cols(D, q):
    """All columns of op q of a downloaded log, as one comparable tuple."""
    nd = D["snap_vc"].shape[0]
    pres = int(D["snap_pres"][q]) if D["snap_pres"] is not None else (1 << nd) - 1
    var = ()
    if D["var_off"] is not None:
        var = tuple(int(x) for x in D["var_data"][int(D["var_off"][q]):int(D["var_off"][q + 1])])
    tx = int(D["op_txid"][q]) if D["op_txid"] is not None else None
    return (int(D["op_meta"][q]), int(D["commit_time"][q]), tuple(int(D["snap_vc"][d, q]) for d in range(nd)),
            pres, tx, int(D["p0"][q]), int(D["p1"][q]), var)


def _key_ops(D, k):
    o0, o1 = int(D["key_off"][k]), int(D["key_off"][k + 1])
    return [(int(D["op_id"][q]), _op_cols(D, q)) for q in range(o0, o1)]


def _oracle_kept_ids(k, ops, thr):
    n, kept = R.prune_ops(len(ops), _tuple(k, ops), thr)
    if kept == [(R.FIRST_OP, 0)] and n == 1:   # the all-pruned quirk (:580-583)
        return None
    return [op[0] for _pos, op in sorted(kept)]


@pytest.mark.parametrize("seed", range(4))
def test_gpu_prune_ops_host_threshold(mat, seed):
    rng = random.Random(7100 + seed)
    n_dc = [1, 3, 5, 8][seed]
    partial = seed >= 2
    n_keys = 48
    keys, types = [], []
    for k in range(n_keys):
        t = randlog.TYPES[k % 5]
        keys.append(randlog.rand_key_ops(rng, t, n_dc, rng.choice([0, 1, 5, 30, 64, 65, 140]), partial=partial,
                                         txids=(seed == 1)))
        types.append(t)
    log = HostLog(n_dc, keys, key_types=types)
    s0 = mat.store(log)
    mask = np.zeros(n_keys, np.uint8)
    thr_vc = np.zeros((n_dc, n_keys), np.uint64)
    thr_pres = np.zeros(n_keys, np.uint32)
    thr = {}
    for k, ops in enumerate(keys):
        if rng.random() < 0.8:
            mask[k] = 1
            hi = ops[-1].commit_time if ops else 30
            c = {d: int(rng.randint(0, hi + 10)) for d in range(n_dc) if not (partial and rng.random() < 0.2)}
            if rng.random() < 0.15:
                c = {d: hi + 100 for d in range(n_dc)}   # prunes everything
            thr[k] = c
            for d, v in c.items():
                thr_vc[d, k] = v
                thr_pres[k] |= 1 << d
    s1, flags = s0.update(prune=(mask, thr_vc, thr_pres))
    try:
        D0, D1 = s0.download(), s1.download()
        assert int(D1["key_off"][-1]) == len(D1["op_meta"])
        for k, ops in enumerate(keys):
            got = _key_ops(D1, k)
            old = dict(_key_ops(D0, k))
            if not mask[k]:
                assert got == _key_ops(D0, k), k
                assert flags[k] & abi.AM_GC_PRUNED_ALL == 0
                continue
            ref = _oracle_kept_ids(k, ops, thr[k])
            if ref is None:
                assert got == [] and flags[k] & abi.AM_GC_PRUNED_ALL, (k, got)
                continue
            assert [i for i, _ in got] == ref, (k, thr[k])
            assert all(cols == old[i] for i, cols in got), k
            assert not flags[k] & abi.AM_GC_PRUNED_ALL
            assert D1["key_type"][k] == D0["key_type"][k]
        # reads through the rebuilt log equal reads of the oracle on the pruned tuples
        reads, refs = [], []
        for k, ops in enumerate(keys):
            if not ops or types[k] not in (abi.AM_PN, abi.AM_LWW):
                continue
            clock = {d: ops[-1].commit_time + 20 for d in range(n_dc)}
            reads.append(Read(k, types[k], clock))
            ids = [i for i, _ in _key_ops(D1, k)]
            kept = [ops[i - 1] for i in ids]
            resp = R.SnapshotGetResponse(ops_list=_tuple(k, kept, ids) if kept else [], number_of_ops=len(kept),
                                         materialized_snapshot=R.MatSnapshot(0, R.crdt_new(types[k])),
                                         snapshot_time=R.IGNORE, is_newest_snapshot=True)
            refs.append(R.materialize(types[k], R.IGNORE, dict(clock), resp) if kept else None)
        hb = mat.read_batch(s1, reads)
        for i, (rd, ref) in enumerate(zip(reads, refs)):
            g = hb.result(i)
            if ref is None:
                assert g[0] == "ok" and g[1] == randlog.canon_state(rd.type, R.crdt_new(rd.type)), (rd, g)
            else:
                assert g[0] == "ok" and g[1] == randlog.canon_state(rd.type, ref[1]) and g[2] == ref[2] and g[5] == ref[5], (rd, g, ref)
    finally:
        s1.close()
        s0.close()


def test_gpu_op_insert_ids_and_trigger(mat):
    """Appends get NewId = OpCounter + 1, ... (op_insert_gc/3, :630), the counter survives a
    GC that prunes every op, and AM_GC_TRIGGER marks NewId rem OPS_THRESHOLD == 0 (:635)."""
    rng = random.Random(77)
    n_dc, n_keys = 3, 24
    types = [randlog.TYPES[k % 5] for k in range(n_keys)]
    keys = [randlog.rand_key_ops(rng, types[k], n_dc, rng.choice([0, 3, 48, 49, 50, 99])) for k in range(n_keys)]
    store = mat.store(HostLog(n_dc, keys, key_types=types))
    counters = [len(o) for o in keys]
    D = store.download()
    expect = [_key_ops(D, k) for k in range(n_keys)]
    try:
        for rnd in range(4):
            if rnd == 2:   # prune every op of the even keys: the counter must survive
                mask = np.array([1 if k % 2 == 0 else 0 for k in range(n_keys)], np.uint8)
                big = np.full((n_dc, n_keys), 2**62, np.uint64)
                pres = np.full(n_keys, (1 << n_dc) - 1, np.uint32)
                nxt, flags = store.update(prune=(mask, big, pres))
                for k in range(n_keys):
                    if mask[k]:
                        assert flags[k] & abi.AM_GC_PRUNED_ALL, k
                        expect[k] = []
                store.close()
                store = nxt
            new = []
            for k in range(n_keys):
                t0 = (keys[k][-1].commit_time if keys[k] else 10) + 1000 * (rnd + 1)
                new.append(randlog.rand_key_ops(rng, types[k], n_dc, rng.choice([0, 1, 2, 7, 50, 70]), t0=t0)
                           if rng.random() < 0.8 else [])
            nlog = HostLog(n_dc, new, key_types=types)
            nxt, flags = store.update(new_log=nlog)
            ND = mat.store(nlog).download()
            D1 = nxt.download()
            for k in range(n_keys):
                c, n = counters[k], len(new[k])
                trig = any((c + j) % abi.AM_OPS_THRESHOLD == 0 for j in range(1, n + 1))
                assert bool(flags[k] & abi.AM_GC_TRIGGER) == trig, (k, c, n)
                appended = [(c + 1 + j, cols) for j, (_i, cols) in enumerate(_key_ops(ND, k))]
                expect[k] = expect[k] + appended
                assert _key_ops(D1, k) == expect[k], (rnd, k)
                # the oracle's op_insert_gc assigns the same ids
                t = _tuple(k, [], [], counter=c)
                st = R.VnodeState(ops_cache={k: t})
                ids = []
                for op in new[k]:
                    R.op_insert_gc(k, randlog.payload_term(op, key=k), st)
                    ids.append(st.ops_cache[k].element(3))
                assert ids == [i for i, _ in appended], k
                counters[k] = c + n
            store.close()
            store = nxt
    finally:
        store.close()


def test_gpu_gc_from_snapshot_cache(mat):
    """snapshot_insert_gc/4 end to end: cache reads fill the device snapshot cache; the forced
    GC (am_snapcache_gc_threshold) truncates every dict to its newest SNAPSHOT_MIN snapshots and
    their vectorclock:min prunes the log; later reads through the pruned log with the same
    cache -- low clocks (the cold path) included -- match the oracle."""
    rng = random.Random(4242)
    n_dc, n_keys = 3, 32
    types = [abi.AM_PN if k % 2 == 0 else abi.AM_LWW for k in range(n_keys)]
    keys = [randlog.rand_key_ops(rng, types[k], n_dc, rng.choice([0, 10, 60, 150, 300])) for k in range(n_keys)]
    store = mat.store(HostLog(n_dc, keys, key_types=types))
    cache = mat.snapshot_cache(store, n_keys)
    st = R.VnodeState()
    for k, ops in enumerate(keys):
        if ops:
            st.ops_cache[k] = _tuple(k, ops)
    hi = [ops[-1].commit_time if ops else 20 for ops in keys]

    def read_round(q_lo, q_hi):
        reads = []
        for k in range(n_keys):
            c = int(10 + (hi[k] - 10) * rng.uniform(q_lo, q_hi))
            reads.append(Read(k, types[k], {d: c + rng.randint(0, 3) for d in range(n_dc)}))
        got = cache.read(reads)
        for i, rd in enumerate(reads):
            try:
                ref = R.internal_read(rd.key, rd.type, dict(rd.clock), R.IGNORE, False, st)
            except R.LogColdPath:
                assert got.result(i) == ("error", abi.AM_ERR_COLD_PATH)
                continue
            g = got.result(i)
            assert g[0] == "ok" and g[1] == randlog.canon_state(rd.type, ref[1]), (rd, g, ref)

    try:
        for rnd in range(6):
            read_round(0.1 * rnd, 0.1 * rnd + 0.25)
        D0 = store.download()
        s1, flags = store.update(prune=cache)
        D1 = s1.download()
        for k, ops in enumerate(keys):
            if k not in st.snapshot_cache or st.snapshot_cache[k][1] == 0:
                assert _key_ops(D1, k) == _key_ops(D0, k)
                continue
            sub = R.vo_sublist(st.snapshot_cache[k], 1, R.SNAPSHOT_MIN)
            thr = R.gc_threshold(sub)
            st.snapshot_cache[k] = sub  # snapshot_insert_gc stores PrunedSnapshots (:536)
            t = st.ops_cache.get(k)
            if t is None:
                assert _key_ops(D1, k) == []
                continue
            n = t.element(2)[0]
            cur = [t.element(R.FIRST_OP + i) for i in range(n)]
            new_len, kept = R.prune_ops(n, t, thr)
            if kept == [(R.FIRST_OP, 0)] and new_len == 1:
                assert _key_ops(D1, k) == [] and flags[k] & abi.AM_GC_PRUNED_ALL
                kept_ops = []
            else:
                kept_ops = [op for _pos, op in sorted(kept)]
                assert [i for i, _ in _key_ops(D1, k)] == [i for i, _ in kept_ops], k
            assert len(cur) == n
            st.ops_cache[k] = R.OpsTuple(k, len(kept_ops), t.element(2)[1], t.element(3), kept_ops)
        cache.store = s1
        read_round(0.0, 0.3)  # below the kept snapshots: the cold path, on both sides
        for rnd in range(6, 11):
            read_round(0.1 * rnd, 0.1 * rnd + 0.3)
        store.close()
        store = s1
    finally:
        cache.close()
        store.close()


def test_gpu_load_ops_bulk_rebuild(mat):
    """load_from_log_to_tables/2 -> load_ops/2 (src/materializer_vnode.erl:288-319): replaying a
    partition's committed ops through op_insert_gc/3 -- ids 1..n per key, and the GC read
    every 50 ids / on a full tuple (snapshot cached, ops pruned, ListLen resized) -- against
    the oracle's replay (R.op_insert_gc per op): the same ops cache and snapshot cache key by
    key, then the same reads."""
    from tests.test_gpu_vnode import KeyGen, compare_state, _placeholder
    rng = random.Random(99)
    n_dc, n_keys = 4, 40
    types = [randlog.TYPES[k % 5] for k in range(n_keys)]
    keys = [KeyGen(rng, types[k], n_dc, 10 + k).ops(rng.choice([0, 1, 9, 64, 130, 260])) for k in range(n_keys)]
    vn = mat.load_ops(n_dc, keys, key_types=types)
    st = R.VnodeState()
    dead = set()
    for k in range(n_keys):
        for op in keys[k]:
            if _placeholder(st, k):  # a GC read pruned every op: the reference crashes on its placeholder
                dead.add(k)
                break
            R.op_insert_gc(k, randlog.payload_term(op, key=k), st)
    try:
        live = [k for k in range(n_keys) if k not in dead and not _placeholder(st, k)]
        compare_state(vn, st, {k: k for k in live}, types, {d: d for d in range(n_dc)})
        assert sum(1 for k in live if len(keys[k]) >= 130) >= 8  # keys that went through GC reads
        reads = [Read(k, types[k], {d: (keys[k][-1].commit_time if keys[k] else 30) + 3 for d in range(n_dc)})
                 for k in live]
        got = vn.read(reads, set_capacity=[4096] * len(reads))
        for i, rd in enumerate(reads):
            ref = R.internal_read(rd.key, rd.type, dict(rd.clock), R.IGNORE, False, st)
            assert got.result(i)[0] == "ok" and got.result(i)[1] == randlog.canon_state(rd.type, ref[1]), i
    finally:
        vn.close()
