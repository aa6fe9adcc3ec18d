"""Caller-side read batching (antidote_amd.readbatch.PartitionedReader): read_objects fan-out
(src/clocksi_interactive_coord.erl:732-747) grouped into one am_materialize batch per
partition.  Bar: every object's result equals the oracle's materialize/4 on that key's log,
in request order, with keys spread over partitions by get_key_partition/1."""
import random

import pytest

from antidote_amd import abi
from antidote_amd.oplog import Read
from tests import randlog

pytestmark = pytest.mark.gpu


def test_gpu_read_objects_partitioned():
    from antidote_amd.materializer import Materializer
    from antidote_amd.readbatch import PartitionedReader
    rng = random.Random(515)
    n_dc, n_part = 3, 8
    keys = rng.sample(range(-5000, 5000), 120)
    objects = {}
    for key in keys:
        t = rng.choice(randlog.TYPES)
        objects[key] = (t, randlog.rand_key_ops(rng, t, n_dc, rng.choice([0, 1, 6, 40, 100])))
    mat = Materializer(0)
    rd = PartitionedReader(mat, n_part, n_dc, objects)
    try:
        assert {rd.partition_of(k) for k in keys} == set(range(n_part))
        assert all(rd.partition_of(k) == abs(k) % n_part for k in keys)
        for _ in range(4):
            req = rng.sample(keys, 50)
            clock = {d: rng.randint(20, 250) for d in range(n_dc)}
            got = rd.read_objects([(k, objects[k][0]) for k in req], clock)
            for k, g in zip(req, got):
                t, ops = objects[k]
                assert g == randlog.ref_materialize(t, ops, Read(0, t, dict(clock))), (k, g)
    finally:
        rd.close()
        mat.close()
