"""Caller-side read batching through the C-ABI (am_read_objects_submit / am_ticket_wait):
a transaction's read_objects fan-out (src/clocksi_interactive_coord.erl:732-747) over the
partitions one GPU owns -- keys placed by get_key_partition/1 -- is ONE asynchronous
internal_read/7 batch on a vnode whose key space concatenates the partitions'.  Bar: every
object's result, in request order, equals the oracle's VnodeState (op_insert_gc/3 replay +
internal_read/7 in request order, snapshot cache included); two transactions in flight at
once on disjoint keys give the same results as run one after the other."""
import random

import pytest

from antidote_amd import abi
from antidote_amd.oplog import Read
from oracle import ref_materializer as R
from tests import randlog
from tests.test_gpu_vnode import KeyGen, _placeholder

pytestmark = pytest.mark.gpu


def _check(got, reqs, clock, st, dead):
    for (key, t), g in zip(reqs, got):
        if _placeholder(st, key):
            dead.add(key)
        if key in dead:
            continue
        try:
            ref = R.internal_read(key, t, dict(clock), R.IGNORE, False, st)
        except R.LogColdPath:
            assert g == ("error", abi.AM_ERR_COLD_PATH), (key, g)
            continue
        assert g[0] == "ok" and g[1] == randlog.canon_state(t, ref[1]), (key, g, ref)


def test_gpu_read_objects_partitioned():
    from antidote_amd.materializer import Materializer
    from antidote_amd.readbatch import PartitionedReader
    rng = random.Random(515)
    n_dc, n_part = 3, 8
    keys = rng.sample(range(-5000, 5000), 120)
    objects, gens = {}, {}
    for key in keys:
        t = rng.choice(randlog.TYPES)
        gens[key] = KeyGen(rng, t, n_dc, 10)
        objects[key] = (t, gens[key].ops(rng.choice([0, 1, 6, 40, 100])))
    st = R.VnodeState()
    dead = set()
    for key in keys:
        for op in objects[key][1]:
            if _placeholder(st, key):
                dead.add(key)
                break
            R.op_insert_gc(key, randlog.payload_term(op, key=key), st)
    mat = Materializer(0)
    rd = PartitionedReader(mat, n_part, n_dc, objects)
    try:
        assert {rd.partition_of(k) for k in keys} == set(range(n_part))
        assert all(rd.partition_of(k) == abs(k) % n_part for k in keys)
        hi = max(g.clock for g in gens.values())
        for rnd in range(6):
            clock = {d: rng.randint(hi // 2, hi + 10) for d in range(n_dc)}
            if rnd % 2 == 0:  # one transaction, repeated keys across partitions
                req = [(k, objects[k][0]) for k in rng.choices(keys, k=60)]
                _check(rd.read_objects(req, clock), req, clock, st, dead)
            else:  # two transactions in flight on disjoint keys
                ks = rng.sample(keys, 80)
                ra = [(k, objects[k][0]) for k in ks[:40]]
                rb = [(k, objects[k][0]) for k in ks[40:]]
                pa, pb = rd.submit(ra, clock), rd.submit(rb, clock)
                gb, ga = pb.result(), pa.result()
                _check(ga, ra, clock, st, dead)
                _check(gb, rb, clock, st, dead)
        # a request outside its partition is rejected per read, not per call
        from antidote_amd.oplog import HostBatch
        import ctypes
        import numpy as np
        hb = HostBatch(n_dc, [Read(10**6, abi.AM_PN, {0: 5})], [1])
        b, r = hb.structs()
        parts = np.zeros(1, np.uint32)
        abi.check(mat.L.am_read_objects_host(rd.vnode.handle, n_part, rd.part_key_base.ctypes.data, parts.ctypes.data,
                                             ctypes.byref(b), ctypes.byref(r)), "am_read_objects_host")
        assert hb.result(0) == ("error", abi.AM_ERR_INVALID)
    finally:
        rd.close()
        mat.close()


def test_gpu_read_objects_dropped_and_closed():
    """A PendingRead dropped before result() waits for its worker (the worker writes into its
    host buffers until am_ticket_wait), and closing the reader with reads in flight waits for
    them before the vnode goes away."""
    import gc

    from antidote_amd.materializer import Materializer
    from antidote_amd.readbatch import PartitionedReader
    rng = random.Random(616)
    n_dc, n_part = 2, 4
    keys = list(range(40))
    objects = {}
    for key in keys:
        g = KeyGen(rng, randlog.TYPES[key % 4], n_dc, 10)
        objects[key] = (randlog.TYPES[key % 4], g.ops(rng.choice([1, 8, 60])))
    mat = Materializer(0)
    rd = PartitionedReader(mat, n_part, n_dc, objects)
    try:
        clock = {d: 10 ** 6 for d in range(n_dc)}
        req = [(k, objects[k][0]) for k in keys]
        ref = rd.read_objects(req, clock)
        for _ in range(4):
            p = rd.submit(req, clock)
            del p
            gc.collect()
        assert not list(rd._pending)
        # the dropped reads ran (through the snapshot cache): a repeat of the first read now
        # serves every key from its cached snapshot, the values unchanged
        assert [g[:2] for g in rd.read_objects(req, clock)] == [g[:2] for g in ref]
        rd.submit(req, clock), rd.submit(req, clock)  # left in flight
    finally:
        rd.close()
        mat.close()
