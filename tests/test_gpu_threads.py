"""One am_ctx shared by concurrent callers (a partition's READ_CONCURRENCY read servers,
include/antidote.hrl:28; src/clocksi_readitem_server.erl:195): threads issue host batches
(am_materialize_host, am_snapcache_read_host, am_vnode_read_host) on the same context at once
-- ctypes releases the GIL during the call -- and every result equals the same batch run
alone.  The context serializes its callers (am_ctx.mu), so no scratch slot is shared."""
import random
import threading

import pytest

from antidote_amd import abi
from antidote_amd.oplog import HostLog, Read
from tests import randlog

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mat():
    from antidote_amd.materializer import Materializer
    m = Materializer(0)
    yield m
    m.close()


def test_gpu_concurrent_callers_one_ctx(mat):
    rng = random.Random(31)
    n_dc, n_keys = 3, 64
    types = [randlog.TYPES[k % 5] for k in range(n_keys)]
    keys = [randlog.rand_key_ops(rng, types[k], n_dc, rng.choice([0, 5, 40, 200, 700])) for k in range(n_keys)]
    store = mat.store(HostLog(n_dc, keys, key_types=types))
    hi = [k[-1].commit_time if k else 20 for k in keys]
    batches = []
    for _ in range(24):
        ks = rng.sample(range(n_keys), 40)
        batches.append([Read(k, types[k], {d: rng.randint(0, hi[k] + 5) for d in range(n_dc)}) for k in ks])
    expect = [[mat.read_batch(store, b, [4096] * len(b)).result(i) for i in range(len(b))] for b in batches]
    got = [None] * len(batches)
    errors = []

    def worker(ix):
        try:
            for j in ix:
                hb = mat.read_batch(store, batches[j], [4096] * len(batches[j]))
                got[j] = [hb.result(i) for i in range(len(batches[j]))]
        except Exception as e:  # surfaced below
            errors.append(e)

    threads = [threading.Thread(target=worker, args=(list(range(t, len(batches), 8)),)) for t in range(8)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(120)
    try:
        assert not errors, errors
        assert got == expect
    finally:
        store.close()


def test_gpu_concurrent_vnode_and_materialize(mat):
    """A vnode's inserts (write-triggered GC) and reads on one thread while plain
    materializations run on four others: the vnode's reads equal the same sequence run alone
    (with GC the values follow op_insert_gc's snapshots, not the full log's, so the alone-run
    is the expectation) and the plain reads keep their single-threaded values."""
    rng = random.Random(32)
    n_dc, n_keys = 2, 16
    types = [randlog.TYPES[k % 5] for k in range(n_keys)]
    keys = [randlog.rand_key_ops(rng, types[k], n_dc, rng.choice([3, 60, 120])) for k in range(n_keys)]
    store = mat.store(HostLog(n_dc, keys, key_types=types))
    hi = [k[-1].commit_time if k else 20 for k in keys]
    reads = [Read(k, types[k], {d: hi[k] + 5 - 3 * j for d in range(n_dc)}) for j in range(2) for k in range(n_keys)]
    caps = [4096] * len(reads)
    expect = mat.read_batch(store, reads, caps)
    exp = [expect.result(i) for i in range(len(reads))]

    def vnode_run():
        vn = mat.vnode(n_dc, n_keys)
        try:
            vn.insert(keys, types)
            out = []
            for j in range(5):
                hb = vn.read(reads, should_gc=[(i + j) % 7 == 0 for i in range(len(reads))], set_capacity=caps)
                out.append([hb.result(i) for i in range(len(reads))])
            return out, [vn.key_info(k) for k in range(n_keys)], [vn.snapshots(k, types[k]) for k in range(n_keys)]
        finally:
            vn.close()

    alone = vnode_run()
    errors, got = [], []

    def plain():
        try:
            for _ in range(20):
                hb = mat.read_batch(store, reads, caps)
                assert [hb.result(i) for i in range(len(reads))] == exp
        except Exception as e:
            errors.append(e)

    def vnode():
        try:
            got.append(vnode_run())
        except Exception as e:
            errors.append(e)

    threads = [threading.Thread(target=plain) for _ in range(4)] + [threading.Thread(target=vnode)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(120)
    try:
        assert not errors, errors
        assert got and got[0] == alone
    finally:
        store.close()
