#!/usr/bin/env python3
"""Bench: CRDT ops materialized/sec (whole node) + % of HBM peak, MI355X.

One step = one batched snapshot read of every key this GPU owns:
  1. GST: am_gst_local_min over this GPU's partition stable clocks -> RCCL min
     all-reduce over all ranks (am_gst_allreduce) -> am_gst_finalize; the stable
     snapshot lands in HBM and is the read's MinSnapshotTime (as a ClockSI
     transaction reads at the GST, src/clocksi_interactive_coord.erl:907-912);
  2. am_materialize of all keys at that snapshot (clocksi_materializer:materialize/4
     per key, fresh base: the first read of each key).
Workload (BASELINE.json configs[1], "C2"): antidote_crdt_register_lww, 1M keys x 256
ops per GPU, 3-DC vectorclocks, synthetic counter-based logs generated in HBM.
Weak scaling: each rank owns its own 1M keys (keys shard by riak_core partition:
partition = key mod 64, GPU = partition mod N), so value = N * 256M ops / step time.

Launch: python bench.py [--gpus 1 --steps K --warmup W]; for N > 1 under
torch.distributed.run (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_ADDR from the env).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from antidote_amd import abi  # noqa: E402
from antidote_amd.devbatch import DeviceReads, materialize  # noqa: E402
from antidote_amd.materializer import Materializer  # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
N_PARTITIONS = 64          # riak_core ring for the multi-GPU layout

CONFIGS = {
    # name: (type, n_dc, keys per GPU, ops per key, q)
    "c2": (abi.AM_LWW, 3, 1 << 20, 256, 0.75),
    "c1": (abi.AM_PN, 1, 10000, 64, 0.75),
}


def bytes_per_op(type_: int, n_dc: int, packed: bool = True) -> int:
    """Algorithmic HBM bytes read per op by the materialize kernel.
    Packed view (am_pack.hip): ct_meta 8 + snapshot deltas 4*D + payload (PN 8, LWW 16);
    full view: op_meta 1 + commit_time 8 + snapshot_time 8*D + payload."""
    payload = 16 if type_ == abi.AM_LWW else 8
    return (8 + 4 * n_dc + payload) if packed else (1 + 8 + 8 * n_dc + payload)


def bytes_per_key(type_: int, n_dc: int) -> int:
    """Per read: key index 8 + type 1 + key_off 8 + key_type 1 (inputs) + outputs status 4,
    new_last_op 8, last_ct 8*D, last_ct_pres 4, last_ct_ignore 1, is_new_ss 1, count 4,
    flags 1, value (PN 8; LWW 8+8+1)."""
    val = 17 if type_ == abi.AM_LWW else 8
    return 8 + 1 + 8 + 1 + 4 + 8 + 8 * n_dc + 4 + 1 + 1 + 4 + 1 + val


def synth_params(type_, n_dc, n_keys, n_ops, key_base):
    p = abi.am_synth_params()
    p.seed, p.n_keys, p.ops_per_key, p.n_dc, p.type, p.key_base, p.max_lag = (0x5EED + 2, n_keys, n_ops, n_dc,
                                                                               type_, key_base, 8)
    return p


def cpu_baseline(p, q, budget_s=10.0, sample_keys=100_000):
    """The C restatement (oracle/am_oracle.c, a port of clocksi_materializer) on the host
    cores, on a bounded sample of the same workload.  Rank 0, N=1 only."""
    sys.path.insert(0, HERE)
    from antidote_amd.oplog import HostBatch, HostLog, Read
    from oracle import amo
    import threading

    nk = min(sample_keys, p.n_keys)
    n_ops = nk * p.ops_per_key
    log = HostLog.__new__(HostLog)
    log.n_dc, log.n_keys, log.n_ops, log.n_var, log.has_var = p.n_dc, nk, n_ops, 0, False
    log.key_off = np.zeros(nk + 1, np.uint64)
    log.key_type = np.zeros(nk, np.uint8)
    log.key_flags = log.key_id_base = log.snap_pres = log.op_txid = log.op_id = None
    log.op_meta = np.zeros(n_ops, np.uint8)
    log.commit_time = np.zeros(n_ops, np.uint64)
    log.snap_vc = np.zeros((p.n_dc, n_ops), np.uint64)
    log.p0 = np.zeros(n_ops, np.uint64)
    log.p1 = np.zeros(n_ops, np.uint64)
    log.var_off = log.var_data = None
    s = log.as_struct()
    abi.check(abi.lib().am_synth_host(ctypes.byref(p), 0, nk, ctypes.byref(s)), "am_synth_host")
    clock = (ctypes.c_uint64 * p.n_dc)()
    abi.lib().am_synth_read_clock(ctypes.byref(p), q, clock)
    hb = HostBatch(p.n_dc, [Read(k, p.type, {d: clock[d] for d in range(p.n_dc)}) for k in range(nk)])
    b, r = hb.structs()
    L = amo.lib()
    threads = max(1, min(16, os.cpu_count() or 1))
    step = (nk + threads - 1) // threads

    def one_pass():
        ts = [threading.Thread(target=L.amo_materialize_range,
                               args=(ctypes.byref(s), ctypes.byref(b), i, min(nk, i + step), ctypes.byref(r)))
              for i in range(0, nk, step)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()

    one_pass()  # warm (page faults)
    t0 = time.perf_counter()
    passes = 0
    while True:
        one_pass()
        passes += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": passes * n_ops / dt, "unit": "ops/s", "cores": threads, "kind": "port",
            "sample": f"{nk} keys x {p.ops_per_key} ops of the same workload, {passes} passes in {dt:.1f}s, "
                      f"C restatement of clocksi_materializer (oracle/am_oracle.c), not BEAM"}


def load_traffic(workload: str):
    """HBM bytes per materialize launch from the committed PMC summary, if it matches."""
    path = os.path.join(HERE, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        if d.get("workload") == workload:
            return d.get("bytes_per_launch")
    except Exception:
        pass
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)
    pg = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)  # control plane only
        pg = dist
    torch.cuda.set_device(local_rank)

    type_, n_dc, n_keys, n_ops, q = CONFIGS[args.config]
    mat = Materializer(local_rank)

    # ---- RCCL communicator for the GST all-reduce (the only data-path collective) ----
    uid = (ctypes.c_char * 128)()
    if rank == 0:
        abi.check(mat.L.am_comm_unique_id(uid), "am_comm_unique_id")
    if pg is not None:
        obj = [bytes(uid)]
        pg.broadcast_object_list(obj, src=0)
        ctypes.memmove(uid, obj[0], 128)
    comm = ctypes.c_void_p()
    # RCCL prints its version banner on stdout; keep stdout for the one JSON line
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        rc = mat.L.am_comm_init(mat.ctx, rank, world, uid, ctypes.byref(comm))
    finally:
        os.dup2(saved, 1)
        os.close(saved)
    abi.check(rc, "am_comm_init")

    # ---- this GPU's op log, generated in HBM ----
    p = synth_params(type_, n_dc, n_keys, n_ops, key_base=rank * n_keys)
    store = mat.synth_store(p)
    dlog = store.device_log()

    # ---- partition stable clocks (GST inputs): this rank owns partitions r, r+N, ... ----
    clock = (ctypes.c_uint64 * n_dc)()
    abi.lib().am_synth_read_clock(ctypes.byref(p), q, clock)
    parts = [pp for pp in range(N_PARTITIONS) if pp % world == rank]
    pvc = np.zeros((len(parts), n_dc), np.uint64)
    for i, pp in enumerate(parts):
        for d in range(n_dc):
            off = 0 if pp == 0 else (np.uint64((pp * 7919 + d * 104729) % 997 + 1))
            pvc[i, d] = np.uint64(clock[d]) + np.uint64(off)
    d_pvc = torch.from_numpy(pvc.view(np.int64)).cuda()
    d_ppres = torch.full((len(parts),), (1 << n_dc) - 1, dtype=torch.int32, device="cuda")
    lanes = torch.zeros(n_dc + 1, dtype=torch.int64, device="cuda")
    last_vc = torch.zeros(n_dc, dtype=torch.int64, device="cuda")
    last_pres = torch.zeros(1, dtype=torch.int32, device="cuda")
    changed = torch.zeros(1, dtype=torch.uint8, device="cuda")

    reads = DeviceReads(n_keys, n_dc, type_, list(clock))
    read_vc, read_pres = reads.read_vc, reads.read_pres   # the GST result is written here

    def step():
        abi.check(mat.L.am_gst_local_min(mat.ctx, n_dc, len(parts), d_pvc.data_ptr(), d_ppres.data_ptr(), None,
                                         lanes.data_ptr()), "gst_local_min")
        abi.check(mat.L.am_gst_allreduce(comm, lanes.data_ptr(), n_dc), "gst_allreduce")
        abi.check(mat.L.am_gst_finalize(mat.ctx, n_dc, lanes.data_ptr(), last_vc.data_ptr(), last_pres.data_ptr(),
                                        0, read_vc.data_ptr(), read_pres.data_ptr(), changed.data_ptr()),
                  "gst_finalize")
        materialize(mat, dlog, reads)

    def barrier():
        torch.cuda.synchronize()
        mat.sync()
        if pg is not None:
            pg.barrier()

    torch.cuda.synchronize()
    for _ in range(args.warmup):
        step()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    dt = time.perf_counter() - t0
    if pg is not None:
        t = torch.tensor([dt], dtype=torch.float64)
        pg.all_reduce(t, op=pg.ReduceOp.MAX)
        dt = float(t.item())

    # sanity: the snapshot read used the GST and every read succeeded
    res = reads.host(0, min(n_keys, 4096))
    assert (res["status"] == 0).all(), "materialize returned errors"
    gst = read_vc.cpu().numpy().view(np.uint64)
    assert [int(x) for x in gst] == [int(clock[d]) for d in range(n_dc)], "GST mismatch"

    # ---- dominant kernel, timed alone with HIP events on the library's stream ----
    kern_iters = max(5, args.steps)
    barrier()
    abi.check(mat.L.am_timer_start(mat.ctx), "timer")
    for _ in range(kern_iters):
        materialize(mat, dlog, reads)
    ms = ctypes.c_float()
    abi.check(mat.L.am_timer_stop(mat.ctx, ctypes.byref(ms)), "timer")
    kern_ms = ms.value / kern_iters
    packed = bool(dlog.ct_meta) and os.environ.get("AM_PACKED", "1") != "0"
    alg_bytes = n_keys * (n_ops * bytes_per_op(type_, n_dc, packed) + bytes_per_key(type_, n_dc))
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9

    total_ops = world * n_keys * n_ops * args.steps
    value = total_ops / dt
    workload = f"{args.config}: antidote_crdt_register_lww, {n_keys} keys x {n_ops} ops per GPU, D={n_dc}" \
        if type_ == abi.AM_LWW else f"{args.config}: antidote_crdt_counter_pn, {n_keys} keys x {n_ops} ops, D={n_dc}"
    out = {
        "metric": "CRDT ops materialized/sec (whole node) + % HBM peak",
        "value": value,
        "unit": "ops/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (counter-based splitmix64 op logs generated in HBM; seed 0x5EED+2)",
        "config": {"workload": workload, "keys_per_gpu": n_keys, "ops_per_key": n_ops, "n_dc": n_dc,
                   "snapshot_quantile": q, "partitions": N_PARTITIONS, "parallelism": f"partition-sharded x{world}",
                   "step": "GST min all-reduce (RCCL) + materialize all keys"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": load_traffic(workload),
                     "kernel": "k_stream" if type_ in (abi.AM_PN, abi.AM_LWW) else "k_sets",
                     "kernel_ms": kern_ms,
                     "alg_bytes_per_launch": alg_bytes,
                     "layout": "packed (ct_meta + int32 snapshot deltas)" if packed else "full"},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(p, q, budget_s=args.cpu_budget)
    if rank == 0:
        print(json.dumps(out), flush=True)
    mat.L.am_comm_destroy(comm)
    store.close()
    mat.close()
    if pg is not None:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
