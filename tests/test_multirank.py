"""world_size-2/4 gloo tests of the multi-GPU layout (CPU): partition ownership, key sharding,
and the GST node-level exchange against the reference's two-level get_min_time + update_stable
(src/meta_data_sender.erl:237-245, 342-356).  The GST path goes through the C ABI's host twins
of the device kernels (am_gst_local_min_host / am_gst_merge_lanes_host / am_gst_finalize_host,
one source with k_gst_local_min / ncclMin / k_gst_finalize in am_gst.hip); gloo carries the
lanes between the processes as RCCL does between GPUs."""
import os
import random
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from oracle import ref_materializer as R

N_PART = 64


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _scenario(seed, world, n_dc=None):
    rng = random.Random(seed)
    n_dc = rng.randint(1, 5) if n_dc is None else n_dc
    table = {}
    for p in range(N_PART):
        r = rng.random()
        if r < 0.05:
            table[p] = R.UNDEFINED
        else:
            table[p] = {d: rng.randint(0, 10**6) for d in range(n_dc) if rng.random() < 0.8}
    return n_dc, table


def _worker(rank, world, port, seed, q):
    import torch
    import torch.distributed as dist

    from antidote_amd import gst
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        stable = None
        snaps = []
        for rnd in range(3):  # three GST rounds: the monotone update_stable across rounds
            n_dc, table = _scenario(seed * 10 + rnd, world, n_dc=1 + seed % 5)
            if stable is None:
                stable = gst.StableHost(n_dc)
            mine = gst.owned_partitions(N_PART, rank, world)
            lanes = gst.local_min_host({p: table[p] for p in mine}, n_dc)   # this node's merge (C ABI)
            got = [None] * world
            dist.all_gather_object(got, lanes.tolist())                     # the RCCL exchange, over gloo
            merged = np.full(n_dc + 1, gst.ABSENT, np.uint64)
            for other in got:
                merged = gst.merge_host(np.asarray(other, np.uint64), merged, n_dc)
            changed, snap = stable.update(merged, gr=(rnd == 2))
            snaps.append((gst.decode(merged, n_dc), changed, snap))
        owned = [0] * N_PART
        for p in gst.owned_partitions(N_PART, rank, world):
            owned[p] = 1
        t = torch.tensor(owned)
        dist.all_reduce(t)
        q.put((rank, snaps, t.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,seed", [(2, 1), (2, 2), (2, 3), (4, 4)])
def test_gst_multi_rank_matches_reference_two_level_merge(world, seed):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, seed, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from antidote_amd import gst
    # reference: per-node local merge, get_min_time over the node dicts, update_stable against
    # the previous round's result (update_func_min), gr broadcast in the last round
    last = {}
    expect = []
    for rnd in range(3):
        n_dc, table = _scenario(seed * 10 + rnd, world, n_dc=1 + seed % 5)
        nodes = {r: R.get_min_time({p: table[p] for p in gst.owned_partitions(N_PART, r, world)})
                 for r in range(world)}
        merged = R.get_min_time(nodes)
        changed, last = R.update_stable(last, merged)
        expect.append((merged, changed, R.gst_gr(last) if rnd == 2 else dict(last)))
    for rank, snaps, owned in res:
        assert snaps == expect, (rank, snaps, expect)
        assert owned == [1] * N_PART          # every partition served by exactly one rank


def test_key_sharding_covers_ranks():
    from antidote_amd import abi, gst
    L = abi.lib()
    for world in (1, 2, 4, 8):
        seen = set()
        for k in range(-500, 500):
            p = L.am_key_partition(k, N_PART)
            rank = p % world
            assert p in gst.owned_partitions(N_PART, rank, world)
            seen.add(rank)
        assert seen == set(range(world))


def test_lane_encoding_roundtrip():
    from antidote_amd import gst
    d = {0: 5, 2: 0, 3: 2**63 + 7}
    assert gst.decode(gst.encode_node(d, 4), 4) == d
    assert gst.decode(gst.encode_node(None, 3), 3) == {}
    with pytest.raises(ValueError):
        gst.encode_node({0: 2**64 - 1}, 1)


def _placement_worker(rank, world, port, q):
    import torch.distributed as dist

    import bench
    from antidote_amd import abi, synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        L = abi.lib()
        cfg = dict(bench.CONFIGS["c4"], n_keys=96, ops=5)
        p = bench.synth_params(cfg, rank, world)
        keys = [int(L.am_synth_key(p, k)) for k in range(p.n_keys)]
        bad = [k for k in keys if L.am_key_partition(k, bench.N_PARTITIONS) % world != rank]
        mine = [pp for pp in range(bench.N_PARTITIONS) if (p.part_mask >> pp) & 1]
        # the rank's log is the global log's slice: key k of this rank == global key keys[k]
        log = synth.host_log(p, 0, p.n_keys)
        g = bench.synth_params(cfg)  # one rank holding every key (identity placement)
        g.n_keys = max(keys) + 1
        same = True
        for k in (0, 1, p.n_keys // 2, p.n_keys - 1):
            a = synth.host_log(p, k, 1)
            b = synth.host_log(g, keys[k], 1)
            same &= bool((a.commit_time == b.commit_time).all() and (a.p0 == b.p0).all()
                         and (a.key_type == b.key_type).all() and (a.snap_vc == b.snap_vc).all())
        out = [None] * world
        dist.all_gather_object(out, (keys, mine))
        q.put((rank, bad, same, out, int(log.n_keys)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_bench_key_placement_follows_partitions(world):
    """bench.py's per-rank logs (am_synth_params.part_mask): rank r holds exactly the keys
    with am_key_partition(key, 64) % N == r, the GST partitions it reduces are the same
    partitions, ranks are disjoint and together hold the first n_keys * N integer keys, and a
    key's ops are the same whichever rank generates them."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_placement_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, bad, same, out, nk in res:
        assert bad == [] and same and nk == 96, (rank, bad, same)
        allkeys = [k for keys, _ in out for k in keys]
        assert sorted(allkeys) == list(range(96 * world))
        for r, (keys, mine) in enumerate(out):
            assert mine == [pp for pp in range(N_PART) if pp % world == r]
            assert {k % N_PART for k in keys} <= set(mine)
