"""In-place ingestion + GC of the touched keys (am_store_reserve / am_store_apply, the vnode's
path: op_insert_gc/3 appends and prune_ops/2 per key, src/materializer_vnode.erl:565-647)
against the whole-store rebuild (am_store_update, itself pinned to the oracle by
test_gpu_gc.py).

Bar: after every round the two stores are equal key by key -- op ids in order, every column of
every op, key type / mixed-type flag, AM_GC_* flags -- and materialize/4 of every key through
both gives identical outputs (every column, every type, mixed-type keys included); a key that
outgrows its room leaves the store untouched (applied = False)."""
import random

import numpy as np
import pytest

from antidote_amd import abi
from antidote_amd.oplog import HostLog, Read
from tests import randlog
from tests.test_gpu_gc import _key_ops

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mat():
    from antidote_amd.materializer import Materializer
    m = Materializer(0)
    yield m
    m.close()


def _same_store(A, B, n_keys):
    for k in range(n_keys):
        assert _key_ops(A, k) == _key_ops(B, k), k
        assert A["key_type"][k] == B["key_type"][k], k
        assert A["key_flags"][k] == B["key_flags"][k], k


def _reads_equal(mat, sa, sb, n_keys, types, n_dc, rng):
    clock = {d: rng.randint(0, 400) for d in range(n_dc)}
    reads = [Read(k, types[k], clock) for k in range(n_keys)]
    ha, hb = mat.read_batch(sa, reads), mat.read_batch(sb, reads)
    for i in range(n_keys):
        assert ha.result(i) == hb.result(i), (i, ha.result(i), hb.result(i))


@pytest.mark.parametrize("seed", range(4))
def test_gpu_apply_matches_rebuild(mat, seed):
    rng = random.Random(9300 + seed)
    n_dc = [1, 3, 5, 8][seed]
    partial = seed == 3
    n_keys = 64
    types = [randlog.TYPES[k % 5] for k in range(n_keys)]
    keys = [randlog.rand_key_ops(rng, types[k], n_dc, rng.choice([0, 1, 5, 20, 40]), partial=partial,
                                 txids=(seed == 2)) for k in range(n_keys)]
    base = mat.store(HostLog(n_dc, keys, key_types=types))
    ref = base
    inp = base.reserve()
    applied_rounds = 0
    try:
        for rnd in range(6):
            touched = sorted(rng.sample(range(n_keys), rng.choice([1, 5, 17])))
            new_ops, new_types = [], []
            for k in touched:
                t = types[k] if rng.random() < 0.9 else randlog.TYPES[rng.randrange(5)]  # some mixed-type keys
                new_types.append(t)
                new_ops.append(randlog.rand_key_ops(rng, t, n_dc, rng.choice([0, 1, 1, 2, 3, 9]), partial=partial,
                                                    txids=(seed == 2)))
            mask = np.zeros(n_keys, np.uint8)
            thr_vc = np.zeros((n_dc, n_keys), np.uint64)
            thr_pres = np.zeros(n_keys, np.uint32)
            for k in touched:
                if rng.random() < 0.5:
                    mask[k] = 1
                    for d in range(n_dc):
                        if not (partial and rng.random() < 0.2):
                            thr_vc[d, k] = rng.randint(0, 300)
                            thr_pres[k] |= 1 << d
            prune = (mask, thr_vc, thr_pres) if mask.any() else None
            # the reference: one whole-store rebuild with the new ops as CSR over every key
            full_ops = [[] for _ in range(n_keys)]
            full_types = list(types)
            for k, ops, t in zip(touched, new_ops, new_types):
                full_ops[k], full_types[k] = ops, t
            nref, fref = ref.update(new_log=HostLog(n_dc, full_ops, key_types=full_types), prune=prune)
            if ref is not base:
                ref.close()
            ref = nref
            before = inp.download()
            ok, fl = inp.apply(touched, new_log=HostLog(n_dc, new_ops, key_types=new_types), prune=prune)
            if ok:
                applied_rounds += 1
                assert [int(x) for x in fl] == [int(fref[k]) for k in touched], (fl, [fref[k] for k in touched])
            else:  # nothing written; the caller's fallback is the rebuild + reserve
                _same_store(inp.download(), before, n_keys)
                nst, _ = inp.update(new_log=HostLog(n_dc, full_ops, key_types=full_types), prune=prune)
                inp.close()
                inp = nst.reserve()
                nst.close()
            _same_store(inp.download(), ref.download(), n_keys)
            _reads_equal(mat, inp, ref, n_keys, full_types, n_dc, rng)
        assert applied_rounds >= 2, applied_rounds  # both paths taken: in place and (a key outgrew its room) rebuild
    finally:
        inp.close()
        if ref is not base:
            ref.close()
        base.close()


def test_gpu_apply_overflow_leaves_store(mat):
    rng = random.Random(9400)
    n_dc, n_keys = 3, 8
    types = [abi.AM_PN, abi.AM_LWW, abi.AM_AWSET, abi.AM_MVREG] * 2
    keys = [randlog.rand_key_ops(rng, types[k], n_dc, 12) for k in range(n_keys)]
    s0 = mat.store(HostLog(n_dc, keys, key_types=types))
    s1 = s0.reserve()
    try:
        before = s1.download()
        _same_store(before, s0.download(), n_keys)
        big = randlog.rand_key_ops(rng, types[2], n_dc, 300)   # far beyond the key's room
        ok, _ = s1.apply([2], new_log=HostLog(n_dc, [big], key_types=[types[2]]))
        assert not ok
        _same_store(s1.download(), before, n_keys)
        ok, _ = s1.apply([0, 5], new_log=HostLog(n_dc, [keys[0][:2], keys[5][:1]], key_types=[types[0], types[5]]))
        assert ok
        after = s1.download()
        assert [i for i, _ in _key_ops(after, 0)] == list(range(1, 15))
        assert [i for i, _ in _key_ops(after, 5)] == list(range(1, 14))
        assert [c for _, c in _key_ops(after, 0)][12:] == [c for _, c in _key_ops(before, 0)][:2]
        for k in (1, 2, 3, 4, 6, 7):
            assert _key_ops(after, k) == _key_ops(before, k), k
    finally:
        s1.close()
        s0.close()


def test_gpu_apply_rejects_bad_keys(mat):
    """am_store_apply takes its touched-key list from the caller: a key outside the store or a
    key listed twice is AM_ERR_INVALID from the C ABI (checked on the device before any kernel
    indexes by it) and from Store.apply (checked on the host), and the store is unchanged; a
    new-op log shaped for another number of keys is AM_ERR_INVALID too, not 'no room'."""
    import ctypes

    from antidote_amd.materializer import _DevBuf
    rng = random.Random(9450)
    n_dc, n_keys = 2, 6
    types = [abi.AM_PN, abi.AM_LWW, abi.AM_AWSET] * 2
    keys = [randlog.rand_key_ops(rng, types[k], n_dc, 4) for k in range(n_keys)]
    s0 = mat.store(HostLog(n_dc, keys, key_types=types))
    s1 = s0.reserve()
    try:
        before = s1.download()
        for bad in ([0, n_keys], [1, 4, 1], [2 ** 40]):
            with pytest.raises(abi.AmError):
                s1.apply(bad)
            kb = _DevBuf.of(mat, np.ascontiguousarray(bad, np.uint64))
            fl = _DevBuf(mat, len(bad))
            ap = ctypes.c_int(7)
            try:
                rc = mat.L.am_store_apply(mat.ctx, s1.handle, len(bad), kb.ptr, None, None, None, None, fl.ptr,
                                          ctypes.byref(ap))
            finally:
                kb.free()
                fl.free()
            assert rc == abi.AM_ERR_INVALID and ap.value == 0, (bad, rc, ap.value)
        with pytest.raises(abi.AmError):   # two new-op key entries for one touched key
            s1.apply([3], new_log=HostLog(n_dc, [keys[3][:1], keys[4][:1]], key_types=[types[3], types[4]]))
        _same_store(s1.download(), before, n_keys)
        ok, _ = s1.apply([3], new_log=HostLog(n_dc, [keys[3][:1]], key_types=[types[3]]))
        assert ok
    finally:
        s1.close()
        s0.close()


def test_gpu_vnode_inserts_in_place(mat):
    """A vnode's steady-state inserts (a few keys per batch, GC triggers included) take the
    in-place path: after the first insert builds the room, batches touching few keys do not
    rebuild the store, and every key's tuple header, op ids and snapshot dict match the oracle's
    VnodeState."""
    from oracle import ref_materializer as R
    from tests.test_gpu_vnode import KeyGen, compare_state
    rng = random.Random(9500)
    n_dc, n_keys = 3, 40
    types = [randlog.TYPES[k % 4] for k in range(n_keys)]
    gens = [KeyGen(rng, types[k], n_dc, 10 + rng.randint(0, 50)) for k in range(n_keys)]
    vn = mat.vnode(n_dc, n_keys)
    st = R.VnodeState()
    try:
        for step in range(10):
            batch = [[] for _ in range(n_keys)]
            for k in (range(n_keys) if step == 0 else rng.sample(range(n_keys), 3)):
                batch[k] = gens[k].ops(3 if step == 0 else rng.choice([1, 2, 30]))
            for k in range(n_keys):
                for op in batch[k]:
                    R.op_insert_gc(k, randlog.payload_term(op, key=k), st)
            vn.insert(batch, types)
            compare_state(vn, st, {k: k for k in range(n_keys)}, types, {d: d for d in range(n_dc)})
        rebuilds, in_place = vn.stats()
        assert rebuilds <= 3 and in_place >= 9, (rebuilds, in_place)
    finally:
        vn.close()


def test_gpu_vnode_grows_key_space(mat):
    """op_insert_gc/3 of a key the ops cache has never seen creates its tuple
    (src/materializer_vnode.erl:624-629): an insert over more keys than the vnode holds grows
    its key space; old keys keep their ops and snapshots, new keys behave as fresh tuples."""
    from oracle import ref_materializer as R
    from tests.test_gpu_vnode import KeyGen, compare_state
    rng = random.Random(9600)
    n_dc = 2
    types = [randlog.TYPES[k % 4] for k in range(30)]
    gens = [KeyGen(rng, types[k], n_dc, 10) for k in range(30)]
    vn = mat.vnode(n_dc, 4)
    st = R.VnodeState()
    try:
        for n in (4, 9, 30):
            batch = [gens[k].ops(rng.choice([1, 3, 55])) for k in range(n)]
            for k in range(n):
                for op in batch[k]:
                    R.op_insert_gc(k, randlog.payload_term(op, key=k), st)
            vn.insert(batch, types[:n])
            assert vn.n_keys == n
            reads = [Read(k, types[k], {d: gens[k].clock + 5 for d in range(n_dc)}) for k in range(n)]
            got = vn.read(reads, set_capacity=[4096] * n)
            for i, rd in enumerate(reads):
                ref = R.internal_read(rd.key, rd.type, dict(rd.clock), R.IGNORE, False, st)
                assert got.result(i)[0] == "ok" and got.result(i)[1] == randlog.canon_state(rd.type, ref[1]), i
            compare_state(vn, st, {k: k for k in range(n)}, types, {d: d for d in range(n_dc)})
    finally:
        vn.close()


def test_gpu_vnode_load_hot_key_beside_short_keys(mat):
    """load_ops/2-style replay of one long log (3,000 ops: a GC read every 50 ids) beside 2,000
    short ones: every GC round after the first is an in-place apply of the keys it touches (the
    hot key), not a whole-store rebuild, and the hot key's tuple matches the oracle's."""
    import time

    from oracle import ref_materializer as R
    from tests.test_gpu_vnode import KeyGen, compare_state
    rng = random.Random(9700)
    n_dc, n_keys = 2, 2001
    types = [abi.AM_PN] * n_keys
    gens = [KeyGen(rng, abi.AM_PN, n_dc, 10) for _ in range(n_keys)]
    batch = [gens[k].ops(3000 if k == 0 else 3) for k in range(n_keys)]
    st = R.VnodeState()
    for k in (0, 1, 2):
        for op in batch[k]:
            R.op_insert_gc(k, randlog.payload_term(op, key=k), st)
    vn = mat.vnode(n_dc, n_keys)
    try:
        t0 = time.perf_counter()
        vn.insert(batch, types)
        dt = time.perf_counter() - t0
        rebuilds, in_place = vn.stats()
        print(f"load: {sum(len(b) for b in batch)} ops, {dt * 1e3:.0f} ms, {rebuilds} rebuilds, {in_place} in place")
        assert in_place >= 100 and rebuilds <= 8, (rebuilds, in_place)
        compare_state(vn, st, {0: 0, 1: 1, 2: 2}, types, {d: d for d in range(n_dc)})
    finally:
        vn.close()


@pytest.mark.parametrize("n_dc", [2, 5])
def test_gpu_apply_escaped_ops(mat, n_dc):
    """Ops escaped from the packed view (a snapshot entry 2^33 us behind: a lagging DC) in a
    store with escape rows, then appended in place (an op written in place reads its escaped
    inputs from the columns, am_op_log.esc_rows): reads match the oracle over the same ops and
    a store built from them (rows for every escaped op)."""
    from oracle import amo
    from antidote_amd.oplog import HostBatch
    rng = random.Random(9500 + n_dc)
    t0 = 1 << 40
    n_keys = 48
    types = [randlog.TYPES[k % 5] for k in range(n_keys)]

    def lag(ops):
        for op in ops:
            if rng.random() < 0.3:
                d = rng.choice([d for d in range(n_dc) if d != op.commit_dc])
                op.snap[d] = t0 - (1 << 33)
        return ops

    keys = [lag(randlog.rand_key_ops(rng, types[k], n_dc, rng.choice([0, 3, 20, 70]), t0=t0)) for k in range(n_keys)]
    base = mat.store(HostLog(n_dc, keys, key_types=types))
    inp = base.reserve()
    try:
        touched = sorted(rng.sample(range(n_keys), 20))
        new_ops = []
        for k in touched:
            last = keys[k][-1].commit_time if keys[k] else t0
            new_ops.append(lag(randlog.rand_key_ops(rng, types[k], n_dc, 1, t0=last)))  # fits the key's room
        ok, _ = inp.apply(touched, new_log=HostLog(n_dc, new_ops, key_types=[types[k] for k in touched]))
        assert ok
        full = [list(ops) for ops in keys]
        for k, ops in zip(touched, new_ops):
            full[k] = full[k] + ops
        flog = HostLog(n_dc, full, key_types=types)
        fresh = mat.store(flog)
        try:
            for q in (0.3, 0.7, 1.0):
                clock = {d: t0 + int(q * 400) for d in range(n_dc)}
                reads = [Read(k, types[k], clock) for k in range(n_keys)]
                ref = amo.materialize(flog, HostBatch(n_dc, reads))
                for st in (inp, fresh):
                    got = mat.read_batch(st, reads)
                    for i in range(n_keys):
                        assert got.result(i) == ref.result(i), (q, i, got.result(i), ref.result(i))
        finally:
            fresh.close()
    finally:
        inp.close()
        base.close()
