#!/usr/bin/env python3
"""Bench: CRDT ops materialized/sec (whole node) + % of HBM peak, MI355X.

One step = one batched snapshot read of every key this GPU owns:
  1. GST: am_gst_local_min over this GPU's partition stable clocks -> RCCL min
     all-reduce over all ranks (am_gst_allreduce) -> am_gst_finalize; the stable
     snapshot lands in HBM and is the read's MinSnapshotTime (as a ClockSI
     transaction reads at the GST, src/clocksi_interactive_coord.erl:907-912);
  2. --base fresh (default): am_materialize of all keys at that snapshot
     (clocksi_materializer:materialize/4 per key, base ignore: the first read of each key);
     --base cached: am_snapcache_read of all keys (materializer_vnode:read/6 ->
     internal_read/7: base snapshot from the device snapshot cache, materialize/4, write-back),
     the cache holding each key's q = 0.5 snapshot (SURVEY.md 8(d)'s cached mode).  The cache
     is rebuilt at q = 0.5 between steps outside the timed region; each step's GST + read is
     timed with HIP events on the library's stream.
  Mixed-type configs (c4, c5) are one mixed batch: the library's planner splits it by type on
  the device.
Default workload: c3 (BASELINE.json configs[2], the largest single-GPU configuration):
antidote_crdt_set_aw, 1M keys x 1024 ops per GPU, 8-DC vectorclocks, synthetic counter-based
logs generated in HBM.  --config c1..c5 selects the other BASELINE.json configs (see CONFIGS).
Weak scaling: each rank owns its own keys (keys shard by riak_core partition:
partition = key mod 64, GPU = partition mod N; rank r's log holds exactly the keys with
am_key_partition(key, 64) % N == r), so value = N * ops per GPU / step time.

Launch: python bench.py [--gpus 1 --steps K --warmup W --config c3 --base fresh]; for N > 1
under torch.distributed.run (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_ADDR from the env).
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

from antidote_amd import abi, synth  # noqa: E402
from antidote_amd.devbatch import DeviceReads, materialize  # noqa: E402
from antidote_amd.materializer import Materializer  # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
N_PARTITIONS = 64          # riak_core ring for the multi-GPU layout
Q = 0.75                   # snapshot quantile: ~75% of each log is in the read's snapshot

# Workloads (BASELINE.json configs), per GPU: weak scaling, each rank owns
# its own keys, so the node-wide totals of C4/C5 are reached at N = 8.
CONFIGS = {
    "c1": dict(type=abi.AM_PN, n_dc=1, n_keys=10000, ops=64, set_cap=0,
               desc="antidote_crdt_counter_pn, 10000 keys x 64 ops, D=1"),
    "c2": dict(type=abi.AM_LWW, n_dc=3, n_keys=1 << 20, ops=256, set_cap=0,
               desc="antidote_crdt_register_lww, 1048576 keys x 256 ops per GPU, D=3"),
    "c3": dict(type=abi.AM_AWSET, n_dc=8, n_keys=1 << 20, ops=1024, set_cap=64,
               desc="antidote_crdt_set_aw, 1048576 keys x 1024 ops per GPU, D=8, 64-element universe"),
    "c4": dict(type=0, n_dc=3, n_keys=8 << 20, ops=16, set_cap=16,
               desc="mixed 40% PN / 20% LWW / 20% AW-set / 20% MV, 8388608 keys x 16 ops per GPU "
                    "(64M keys at 8 GPUs), D=3"),
    # total_ops is the Zipf target BEFORE the hot-key cap: 187267328 is the smallest target (to
    # 4096) whose capped lengths still sum to >= 2^27 (134218704 ops per GPU, 1.07G at 8 GPUs)
    "c5": dict(type=abi.AM_SYNTH_MV_BC, n_dc=16, n_keys=2 << 20, zipf=1.1, total_ops=187267328, hot_cap=1 << 20,
               set_cap=8, desc="MV register + bounded counter (50/50), Zipf s=1.1 key popularity, 2097152 keys / "
                               "134218704 ops per GPU after the 2^20 hot-key cap (16M keys / 1.07G ops at 8 GPUs), "
                               "D=16"),
}


def bytes_per_op(type_: int, n_dc: int, packed: bool = True) -> int:
    """Algorithmic HBM bytes read per op by its materialize kernel.
    Packed view: commit vector 4*D (u32 relative to the key's time base) + payload (PN 8,
    LWW 16, bcounter 16 + op_meta 1; add-wins-set / MV-register effects come from the record
    view, counted per record in workload_bytes; the key's time base 8 B per read).  Full view (logs without the packed view): op_meta 1 + commit_time 8 +
    snapshot_time 8*D + payload (PN 8, LWW 16; AW var_off 8; MV p0 p1 var_off 24; bcounter
    p0 p1 16), variable-length effect words counted separately, 8 B each."""
    if packed:
        return 4 * n_dc + {abi.AM_PN: 8, abi.AM_LWW: 16, abi.AM_AWSET: 0, abi.AM_MVREG: 0, abi.AM_BCOUNTER: 17}[type_]
    payload = {abi.AM_PN: 8, abi.AM_LWW: 16, abi.AM_AWSET: 8, abi.AM_MVREG: 24, abi.AM_BCOUNTER: 16}[type_]
    return 1 + 8 + 8 * n_dc + payload


def bytes_per_vc(n_dc: int, packed: bool = True) -> int:
    """The commit-vector bytes of one op (packed: 4*D; full view: commit_time + 8*D + op_meta)."""
    return 4 * n_dc if packed else 8 + 8 * n_dc + 1


REC_BYTES = 4    # one birth/kill record of the token-group view: rec_g u32 (am_group.hip)
GMASK_BYTES = 8  # one op's group masks (births | effective kills) of the gmask view (am_pack.hip)


def bytes_per_key(type_: int, n_dc: int, set_len: float = 0.0) -> float:
    """Per read: key index 8 + type 1 + key_off 8 + key_type 1 (inputs) + outputs status 4,
    new_last_op 8, last_ct 8*D, last_ct_pres 4, last_ct_ignore 1, is_new_ss 1, count 4,
    flags 1, value (PN 8; LWW 8+8+1; sets: rec_key_off 8 + key_ngrp 4 + set_off 8 +
    set_len 4 + per surviving pair 16 gathered from the group table and 16 written;
    bcounter: set_off 8 + set_len 4 + 16 per orddict entry written, (slot, value))."""
    if type_ == abi.AM_PN:
        val = 8
    elif type_ == abi.AM_LWW:
        val = 17
    elif type_ == abi.AM_BCOUNTER:
        val = 12 + 16 * set_len
    else:
        val = 24 + 32 * set_len
    return 8 + 1 + 8 + 1 + 4 + 8 + 8 * n_dc + 4 + 1 + 1 + 4 + 1 + val


def owned_partitions_mask(rank: int, world: int) -> int:
    """The riak_core partitions (of N_PARTITIONS) rank owns: p % world == rank."""
    return sum(1 << pp for pp in range(N_PARTITIONS) if pp % world == rank)


def synth_params(cfg, rank=0, world=1):
    """This rank's log: exactly the integer keys whose partition am_key_partition(key, 64)
    (= key mod 64, src/log_utilities.erl:60-79) this rank owns -- local key k is the k-th
    of them (am_synth_params.part_mask).  Per-GPU work is fixed (weak scaling)."""
    p = synth.params(cfg["n_keys"], cfg["n_dc"], cfg["type"], ops_per_key=cfg.get("ops", 0),
                     zipf=cfg.get("zipf", 0.0), total_ops=cfg.get("total_ops", 0), hot_cap=cfg.get("hot_cap", 0),
                     esc_ppm=int(round(cfg.get("escape", 0.0) * 1e6)))
    p.part_mask = owned_partitions_mask(rank, world)
    return p


def key_columns(mat, dlog, n_keys):
    """key_off / key_type of the device log, on the host (setup only)."""
    ko = np.empty(n_keys + 1, np.uint64)
    kt = np.empty(n_keys, np.uint8)
    abi.check(mat.L.am_memcpy_d2h(mat.ctx, ko.ctypes.data, dlog.key_off, ko.nbytes), "d2h key_off")
    abi.check(mat.L.am_memcpy_d2h(mat.ctx, kt.ctypes.data, dlog.key_type, kt.nbytes), "d2h key_type")
    return ko, kt


def set_view_bytes(mat, dlog, ko, kt):
    """Bytes of the set effects a read streams: a short grouped key (<= 16 ops from its aligned
    start, <= 32 groups; the lane tier's quad path) ORs one 8-byte group-mask word per op, every
    other grouped key reads its 4-byte records."""
    n = len(kt)
    ng = np.empty(n, np.uint32)
    rko = np.empty(n + 1, np.uint64)
    abi.check(mat.L.am_memcpy_d2h(mat.ctx, ng.ctypes.data, dlog.key_ngrp, ng.nbytes), "d2h key_ngrp")
    abi.check(mat.L.am_memcpy_d2h(mat.ctx, rko.ctypes.data, dlog.rec_key_off, rko.nbytes), "d2h rec_key_off")
    off0, off1 = ko[:-1].astype(np.int64), ko[1:].astype(np.int64)
    nrec = np.diff(rko.astype(np.int64))
    sets = (kt == abi.AM_AWSET) | (kt == abi.AM_MVREG)
    quad = sets & (ng <= 32) & (off1 <= (off0 & ~3) + 16) & bool(dlog.gmask)
    return float((off1 - off0)[quad].sum()) * GMASK_BYTES + float(nrec[~quad].sum()) * REC_BYTES


GRP_MAX_REC = 2048          # include/antidote_mat.h AM_GRP_MAX_REC
BIG_MIN_OPS = GRP_MAX_REC // 2  # AM_BIG_MIN_OPS: an MV key above it reads through the big-read tier
BCWAVE_OPS = 4096           # am_internal.h AM_BCWAVE_OPS: the bounded-counter wave tier's limit


def lag_split(cfg, dlog, index_level) -> bool:
    """Whether this step streams the lag view (am_op_log.lag_ct / lag / key_lag: 4 + 2 D bytes
    of commit vector per op, 4 D of lag bases per read) anywhere: the store has one (D <= 16),
    no zone index (zone-indexed reads keep the packed view), and the config holds set or
    bounded-counter keys (the PN / LWW stream and row tiers keep the packed view)."""
    return (bool(dlog.lag_ct) and cfg["n_dc"] <= 16 and cfg["type"] not in (abi.AM_PN, abi.AM_LWW)
            and index_level == abi.AM_INDEX_NONE)


def lag_keys(cfg, dlog, ko, kt, mat):
    """The keys whose reads stream the lag view, by the tier the planner gives them (am_plan.hip):
    a single-type set config: every key (the split fresh read; the cached wave tier); a mixed
    config: the lane tier's quad reads (at most 16 ops from the aligned start; sets at most 32
    groups), MV keys in the big view (the big-read inclusion pass), bounded-counter reads of
    the row and wave tiers at D > 8 (up to 4096 ops).  The rest (the lanes' longer reads, the
    fresh wave and workgroup set tiers' reads, the PN / LWW row tier, the bounded-counter runs)
    are counted at the packed size."""
    n = len(kt)
    if cfg["type"] in (abi.AM_AWSET, abi.AM_MVREG):
        return np.ones(n, bool)
    off0, off1 = ko[:-1].astype(np.int64), ko[1:].astype(np.int64)
    lens = off1 - off0
    sets = (kt == abi.AM_AWSET) | (kt == abi.AM_MVREG)
    short = off1 <= (off0 & ~3) + 16
    ng = np.zeros(n, np.uint32)
    if dlog.key_ngrp:
        abi.check(mat.L.am_memcpy_d2h(mat.ctx, ng.ctypes.data, dlog.key_ngrp, ng.nbytes), "d2h key_ngrp")
    quad = short & (~sets | ((ng <= 32) & bool(dlog.gmask))) & (kt != abi.AM_BCOUNTER)
    big_mv = (kt == abi.AM_MVREG) & (lens > BIG_MIN_OPS)
    bc_short = (kt == abi.AM_BCOUNTER) & (lens <= BCWAVE_OPS) & (cfg["n_dc"] > 8)
    return quad | big_mv | bc_short


def workload_bytes(cfg, dlog, ko, kt, reads, packed, mat=None, lag=False):
    """Algorithmic bytes of one am_materialize over every key of the store (the layout model:
    what the kernels must stream of this build's HBM layout).  lag: the keys of
    lag_keys stream the lag view's commit vectors instead of the packed ones."""
    lens = np.diff(ko.astype(np.int64))
    records = packed and bool(dlog.rec_key_off)
    total = set_view_bytes(mat, dlog, ko, kt) if records else float(dlog.n_var) * 8
    set_len = reads.set_len.cpu().numpy() if reads.set_len is not None else None
    D = cfg["n_dc"]
    lk = lag_keys(cfg, dlog, ko, kt, mat) if lag else np.zeros(len(kt), bool)
    for t in sorted(set(int(x) for x in np.unique(kt))):
        m = kt == t
        total += float(lens[m].sum()) * bytes_per_op(t, D, packed)
        # lag view: lag_ct 4 + lags 2 D per op instead of 4 D, lag bases 4 D per read
        total += float(lens[m & lk].sum()) * (4 + 2 * D - 4 * D) + float((m & lk).sum()) * 4 * D
        sl = float(set_len[m].mean()) if (set_len is not None and t in (abi.AM_AWSET, abi.AM_MVREG, abi.AM_BCOUNTER)) \
            else 0.0
        total += float(m.sum()) * (bytes_per_key(t, D, sl) + (8 if packed else 0))
    return total


def logical_bytes(cfg, dlog, ko, kt, reads, cached=False):
    """SURVEY.md 8(d)'s byte model, over the reference's per-op record rather than this build's
    layout: B_op = 8 D (snapshot_time) + 8 (commit_time) + 1 (commit DC) + 8 (op id) + P_type
    (PN 8; LWW 16; AW 8 elem + 8 per token + 4 CSR offset; MV 8 value + 8 token + 4 + 8 per
    overridden token; bcounter 2 + 8) and B_key = 8 (op range) + the output (state + 8 D clock
    + 8 new_last_op + 4 count + 1 flags) + (cached reads) the base (state + 8 D clock + 8 last_op).
    Effect words are counted from the log's var_data (AW: 3 + tokens per entry, of which the
    two counts are not payload)."""
    D = cfg["n_dc"]
    lens = np.diff(ko.astype(np.int64))
    n_ops = {t: float(lens[kt == t].sum()) for t in range(1, 6)}
    fixed = 8 * D + 8 + 1 + 8
    total = sum(n_ops.values()) * fixed
    total += n_ops[abi.AM_PN] * 8 + n_ops[abi.AM_LWW] * 16 + n_ops[abi.AM_BCOUNTER] * 10
    total += n_ops[abi.AM_AWSET] * 4 + n_ops[abi.AM_MVREG] * 20   # CSR offsets; MV value + token
    aw_words = float(dlog.n_var) * 8 - n_ops[abi.AM_AWSET] * 16   # AW elem + tokens, MV overridden
    total += max(aw_words, 0.0)
    set_len = reads.set_len.cpu().numpy().astype(np.float64) if reads.set_len is not None else np.zeros(len(kt))
    state = np.where(kt == abi.AM_PN, 8.0, np.where(kt == abi.AM_LWW, 16.0, 16.0 * set_len))
    per_key = 8 + (8 * D + 8 + 4 + 1) + state
    if cached:
        per_key = per_key + 8 * D + 8 + state
    return total + float(per_key.sum())


def cached_bytes(cfg, pre, reads):
    """Extra algorithmic bytes of a cached-base read (am_snapcache_read) per read: the base
    entry (clock 8*D + presence 4 + last_op 8 + value: PN / LWW 17, set pairs 16 each from the
    value pool), the snapshot-cache dict header (count 1 + owner 4), and the write-back of a
    stored snapshot (the same entry sizes, its pairs 16 each into the pool)."""
    nd = cfg["n_dc"]
    ent = 8 * nd + 4 + 8
    n = reads.n
    total = n * (ent + 5)
    base_pairs = float(pre.set_len.sum().item()) if pre.set_len is not None else 0.0
    total += base_pairs * 16 + (0 if pre.set_len is not None else n * 17)
    stored = ((reads.is_new_ss != 0) & (reads.count >= 5)).cpu().numpy()
    n_st = int(stored.sum())
    total += n_st * ent
    if reads.set_len is not None:
        total += float(reads.set_len.cpu().numpy()[stored].sum()) * 16
    else:
        total += n_st * 17
    return total


def cpu_baseline(cfg, p, budget_s=10.0, cached=False):
    """The C restatement (oracle/am_oracle.c, a port of clocksi_materializer) on the host
    cores, on a bounded sample of the same workload (host-regenerated keys).  Rank 0, N=1.
    cached: every read starts from its q = 0.5 result as the base snapshot (materialize/4 with
    a cached base; the snapshot-cache bookkeeping around it is not part of the port)."""
    from antidote_amd.oplog import HostBatch, Read
    from oracle import amo
    import threading

    ops_hint = cfg.get("ops") or max(1, cfg.get("total_ops", 1) // cfg["n_keys"])
    nk = int(min(100_000, p.n_keys, max(2000, 25_000_000 // ops_hint)))
    if cfg.get("zipf"):  # spread the sample over the popularity ranks: 8 equal key ranges
        k0s = [i * (p.n_keys // 8) for i in range(8)]
        per = nk // 8
    else:
        k0s, per = [0], nk
    clock = synth.read_clock(p, Q)
    parts = []
    for k0 in k0s:
        log = synth.host_log(p, k0, per)
        kt = log.key_type[:per]
        reads = [Read(k, int(kt[k]), {d: clock[d] for d in range(p.n_dc)}) for k in range(per)]
        caps = [p.n_dc * p.n_dc + p.n_dc if int(kt[k]) == abi.AM_BCOUNTER else max(cfg["set_cap"], 1) for k in range(per)]
        hb = HostBatch(p.n_dc, reads, caps)
        s = log.as_struct()
        if cached:
            half = synth.read_clock(p, 0.5)
            h0 = HostBatch(p.n_dc, [Read(k, int(kt[k]), {d: half[d] for d in range(p.n_dc)}) for k in range(per)], caps)
            b0, r0 = h0.structs()
            amo.lib().amo_materialize_range(ctypes.byref(s), ctypes.byref(b0), 0, per, ctypes.byref(r0))
            assert (h0.status[:per] == 0).all(), "cpu baseline: q=0.5 reads failed"
            hb.base_ignore[:] = h0.last_ct_ignore
            hb.base_vc[:] = h0.last_ct
            hb.base_pres[:] = h0.last_ct_pres
            hb.base_last_op[:] = h0.new_last_op
            hb.b_v0[:], hb.b_v1[:], hb.b_vflag[:] = h0.v0, h0.v1, h0.vflag
            hb.b_set_off, hb.b_set_len, hb.b_set_a, hb.b_set_b = h0.o_set_off, h0.o_set_len, h0.o_set_a, h0.o_set_b
            hb._h0 = h0
        b, r = hb.structs()
        parts.append((s, b, r, per, int(log.n_ops), log, hb))
    n_ops = sum(x[4] for x in parts)
    L = amo.lib()
    threads = max(1, min(16, os.cpu_count() or 1))

    def one_pass():
        for (s, b, r, n, _, _, _) in parts:
            step = (n + threads - 1) // threads
            ts = [threading.Thread(target=L.amo_materialize_range,
                                   args=(ctypes.byref(s), ctypes.byref(b), i, min(n, i + step), ctypes.byref(r)))
                  for i in range(0, n, step)]
            for t in ts:
                t.start()
            for t in ts:
                t.join()

    def timed(budget):
        t0 = time.perf_counter()
        passes = 0
        while True:
            one_pass()
            passes += 1
            if time.perf_counter() - t0 >= budget:
                break
        return passes, time.perf_counter() - t0

    one_pass()  # warm (page faults)
    passes, dt = timed(budget_s)
    # the same port on ONE thread (single-threaded and all-core), over the first
    # part of the sample (a few seconds)
    s1, b1, r1, n1 = parts[0][0], parts[0][1], parts[0][2], parts[0][3]
    n1 = max(1, min(n1, n1 * 4 // max(1, threads)))
    ops1 = n1 * (parts[0][4] / max(1, parts[0][3]))
    t1 = time.perf_counter()
    p1 = 0
    while True:
        L.amo_materialize_range(ctypes.byref(s1), ctypes.byref(b1), 0, n1, ctypes.byref(r1))
        p1 += 1
        if time.perf_counter() - t1 >= budget_s / 3:
            break
    d1 = time.perf_counter() - t1
    return {"value": passes * n_ops / dt, "unit": "ops/s", "cores": threads, "kind": "port",
            "single_thread": {"value": p1 * ops1 / d1, "cores": 1, "sample": f"{n1} keys (~{int(ops1)} ops)"},
            "sample": f"{len(k0s) * per} keys ({n_ops} ops) of the same workload"
                      f"{' with q=0.5 cached bases' if cached else ''}, {passes} passes in {dt:.1f}s, "
                      f"C restatement of clocksi_materializer (oracle/am_oracle.c), not BEAM"}


def src_sha16() -> str:
    """Hash of the library's kernel and ABI sources (antidote_amd/csrc, include/antidote_mat.h):
    stamps a PMC traffic record with the code it was measured on."""
    import hashlib
    h = hashlib.sha256()
    csrc = os.path.join(HERE, "antidote_amd", "csrc")
    files = sorted(os.path.join(csrc, f) for f in os.listdir(csrc) if f.endswith((".hip", ".h")))
    for f in files + [os.path.join(HERE, "include", "antidote_mat.h")]:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def load_traffic(config: str, workload: str, zone_index: str = "none"):
    """HBM bytes per materialize launch from the committed PMC summary, if it matches the
    workload, the store's zone index AND the library sources this run uses (src_sha16): a
    record taken on other kernels is not reported (traffic null)."""
    path = os.path.join(HERE, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        e = d.get(config, d)
        if (e.get("workload") == workload and e.get("zone_index", "") == zone_index
                and e.get("src_sha16") == src_sha16()):
            return e.get("calibrated_bytes_per_launch", e.get("bytes_per_launch"))
    except Exception:
        pass
    return None


class Step:
    """One config's store and read batch on this rank, with the GST feeding the batch clock."""

    def __init__(self, mat, comm, cfg, rank, world, index_level):
        self.mat, self.cfg = mat, cfg
        n_dc, n_keys, type_ = cfg["n_dc"], cfg["n_keys"], cfg["type"]
        self.p = synth_params(cfg, rank, world)
        t0 = time.perf_counter()
        self.store = mat.synth_store(self.p)   # generation + packed / token-group views + zone index
        mat.sync()
        self.build_s = time.perf_counter() - t0
        self.index_build_ms = None
        if index_level != abi.AM_INDEX_SUMMARIES:
            self.store.index(index_level)
        self.index_level = index_level
        self.dlog = self.store.device_log()
        self.ko, self.kt = key_columns(mat, self.dlog, n_keys)
        self.n_ops = int(self.ko[-1])
        # partition stable clocks (GST inputs): this rank owns partitions r, r+N, ...
        self.clock = synth.read_clock(self.p, Q)
        parts = [pp for pp in range(N_PARTITIONS) if (self.p.part_mask >> pp) & 1]
        pvc = np.zeros((len(parts), n_dc), np.uint64)
        for i, pp in enumerate(parts):
            for d in range(n_dc):
                off = 0 if pp == 0 else (np.uint64((pp * 7919 + d * 104729) % 997 + 1))
                pvc[i, d] = np.uint64(self.clock[d]) + np.uint64(off)
        self.n_parts = len(parts)
        self.d_pvc = torch.from_numpy(pvc.view(np.int64)).cuda()
        self.d_ppres = torch.full((len(parts),), (1 << n_dc) - 1, dtype=torch.int32, device="cuda")
        self.lanes = torch.zeros(n_dc + 1, dtype=torch.int64, device="cuda")
        self.last_vc = torch.zeros(n_dc, dtype=torch.int64, device="cuda")
        self.last_pres = torch.zeros(1, dtype=torch.int32, device="cuda")
        self.changed = torch.zeros(1, dtype=torch.uint8, device="cuda")
        self.types = torch.from_numpy(self.kt.copy()).cuda() if type_ not in range(1, 6) else None
        self.th = type_ if type_ in range(1, 6) else 0
        self.reads = DeviceReads(n_keys, n_dc, self.th, self.clock, set_cap=max(cfg["set_cap"], 1), types=self.types)
        self.comm = comm
        self.cache = None
        self.pre = None

    def reindex(self, level):
        """Rebuild the zone index at `level`; returns its build time (ms, wall clock)."""
        self.mat.sync()
        t0 = time.perf_counter()
        self.store.index(level)
        self.mat.sync()
        ms = (time.perf_counter() - t0) * 1e3
        self.dlog = self.store.device_log()
        self.index_level = level
        return ms

    def gst(self):
        L, ctx, nd = self.mat.L, self.mat.ctx, self.cfg["n_dc"]
        abi.check(L.am_gst_local_min(ctx, nd, self.n_parts, self.d_pvc.data_ptr(), self.d_ppres.data_ptr(), None,
                                     self.lanes.data_ptr()), "gst_local_min")
        abi.check(L.am_gst_allreduce(self.comm, self.lanes.data_ptr(), nd), "gst_allreduce")
        abi.check(L.am_gst_finalize(ctx, nd, self.lanes.data_ptr(), self.last_vc.data_ptr(), self.last_pres.data_ptr(),
                                    0, self.reads.read_vc.data_ptr(), self.reads.read_pres.data_ptr(),
                                    self.changed.data_ptr()), "gst_finalize")

    def read(self):
        materialize(self.mat, self.dlog, self.reads)

    def step(self):
        self.gst()
        self.read()

    # ---- cached mode: read/6 through the device snapshot cache holding q = 0.5 snapshots ----
    def populate(self):
        """The q = 0.5 reads that fill the snapshot cache (each key's first read caches its
        snapshot: is_newest, >= MIN_OP_STORE_SS ops, src/materializer_vnode.erl:469-509)."""
        cfg, mat = self.cfg, self.mat
        if self.pre is None:
            self.pre = DeviceReads(cfg["n_keys"], cfg["n_dc"], self.th, synth.read_clock(self.p, 0.5),
                                   set_cap=max(cfg["set_cap"], 1), types=self.types)
        if self.cache is not None:
            abi.check(mat.L.am_snapcache_destroy(self.cache), "am_snapcache_destroy")
        h = ctypes.c_void_p()
        abi.check(mat.L.am_snapcache_create(mat.ctx, cfg["n_dc"], cfg["n_keys"], ctypes.byref(h)), "am_snapcache_create")
        self.cache = h
        b, r = self.pre.structs()
        abi.check(mat.L.am_snapcache_read(mat.ctx, h, ctypes.byref(self.dlog), ctypes.byref(b), ctypes.byref(r)),
                  "am_snapcache_read (populate)")

    def cached_read(self):
        b, r = self.reads.structs()
        abi.check(self.mat.L.am_snapcache_read(self.mat.ctx, self.cache, ctypes.byref(self.dlog), ctypes.byref(b),
                                               ctypes.byref(r)), "am_snapcache_read")

    def close(self):
        if self.cache is not None:
            self.mat.L.am_snapcache_destroy(self.cache)
            self.cache = None
        self.store.close()


def measure(st: Step, base: str, steps: int, warmup: int, barrier, pg, timed_wall: bool = True):
    """Time `steps` steps of one config (after `warmup`), then the read call alone.  Returns the
    measured figures (max over ranks of the wall time when pg is given)."""
    mat = st.mat

    def stat(reset, which):
        v = ctypes.c_uint64()
        abi.check(mat.L.am_ctx_stat(mat.ctx, which, ctypes.byref(v), 1 if reset else 0), "am_ctx_stat")
        return float(v.value)

    def stats3(reset):
        return np.array([stat(reset, w) for w in (abi.AM_STAT_OPS_SKIPPED, abi.AM_STAT_RECS_SKIPPED,
                                                  abi.AM_STAT_GSUM_WORDS)])

    def event_ms(fn, pre_fn=None):
        if pre_fn is not None:
            pre_fn()
        barrier()
        abi.check(mat.L.am_timer_start(mat.ctx), "timer")
        fn()
        ms_ = ctypes.c_float()
        abi.check(mat.L.am_timer_stop(mat.ctx, ctypes.byref(ms_)), "timer")
        return float(ms_.value)

    if base == "cached":
        def timed_steps(k):
            return sum(event_ms(lambda: (st.gst(), st.cached_read()), st.populate) * 1e-3 for _ in range(k))
        timed_steps(warmup)
        barrier()
        dt = timed_steps(steps)
        barrier()
    else:
        torch.cuda.synchronize()
        for _ in range(warmup):
            st.step()
        barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            st.step()
        barrier()
        dt = time.perf_counter() - t0
    if pg is not None:
        t = torch.tensor([dt], dtype=torch.float64)
        pg.all_reduce(t, op=pg.ReduceOp.MAX)
        dt = float(t.item())
    # sanity: the snapshot read used the GST and every read succeeded
    stt = st.reads.status.cpu().numpy()
    assert (stt == 0).all(), f"materialize returned errors: {np.unique(stt, return_counts=True)}"
    gst_vc = st.reads.read_vc.cpu().numpy().view(np.uint64)
    assert [int(x) for x in gst_vc] == [int(st.clock[d]) for d in range(st.cfg["n_dc"])], "GST mismatch"

    kern_iters = max(5, steps)
    zs = np.zeros(3)  # per launch: ops skipped by the zone index, records skipped, summary words read
    if base == "cached":
        step_ev = [event_ms(lambda: (st.gst(), st.cached_read()), st.populate) for _ in range(steps)]
        kern_ev = []
        for _ in range(kern_iters):
            st.populate()
            stats3(True)
            kern_ev.append(event_ms(st.cached_read))
            zs += stats3(False) / kern_iters
    else:
        step_ev = [event_ms(st.step) for _ in range(steps)]
        stats3(True)
        kern_ev = [event_ms(st.read) for _ in range(kern_iters)]
        zs = stats3(False) / kern_iters
    skipped, rskip, gsw = (float(x) for x in zs)
    kern_ms = float(np.mean(kern_ev))
    cfg = st.cfg
    packed = bool(st.dlog.pk_vc)
    lag = packed and lag_split(cfg, st.dlog, st.index_level)
    alg_bytes = workload_bytes(cfg, st.dlog, st.ko, st.kt, st.reads, packed, mat, lag=lag)
    if base == "cached":
        alg_bytes += cached_bytes(cfg, st.pre, st.reads)
    # the commit vectors of ops whose zone decided them are not streamed, nor the records whose
    # zones' group summaries stood in for them (4 B per record out, 4 B per summary word in)
    alg_bytes -= skipped * ((4 + 2 * cfg["n_dc"]) if lag else bytes_per_vc(cfg["n_dc"], packed))
    alg_bytes += 4.0 * (gsw - rskip)
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    logical = logical_bytes(cfg, st.dlog, st.ko, st.kt, st.reads, cached=base == "cached")
    return {"dt": dt, "steps": steps, "step_ev": step_ev, "kern_ms": kern_ms, "kern_ms_median": float(np.median(kern_ev)),
            "alg_bytes": alg_bytes, "achieved": achieved, "logical": logical, "skipped": skipped, "rskip": rskip,
            "gsw": gsw, "packed": packed}


def summary(st: Step, m, world: int, label: str):
    """A compact record of one measured config (secondary / indexed lines)."""
    ops = world * st.n_ops
    return {"workload": label, "ops_per_gpu": st.n_ops, "ms_per_step": m["dt"] / m["steps"] * 1e3,
            "ops_per_s": ops * m["steps"] / m["dt"],
            "step_ms_hip_events_median": float(np.median(m["step_ev"])), "kernel_ms": m["kern_ms"],
            "kernel_ms_median": m["kern_ms_median"], "alg_bytes_per_launch": m["alg_bytes"],
            "roofline_frac": m["achieved"] / HBM_PEAK_GBS,
            "logical_frac_of_peak": m["logical"] / (m["kern_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "ops_skipped_per_launch": m["skipped"], "records_skipped_per_launch": m["rskip"],
            "gsum_words_per_launch": m["gsw"], "zone_index": INDEX_NAMES[st.index_level],
            "store_build_s": st.build_s}


INDEX_NAMES = {abi.AM_INDEX_NONE: "none", abi.AM_INDEX_ZONES: "zones (bounds only)",
               abi.AM_INDEX_EXACT: "zones + exact marks", abi.AM_INDEX_SUMMARIES: "zones + exact marks + group summaries"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--base", default="fresh", choices=["fresh", "cached"],
                    help="fresh: base ignore (first read); cached: base from the snapshot cache at q = 0.5")
    ap.add_argument("--index", default="none", choices=["none", "zones", "exact", "summaries"],
                    help="zone index of the headline store (am_store_index); the headline streams every op "
                         "(none) unless asked otherwise")
    ap.add_argument("--escape", type=float, default=0.0,
                    help="fraction of ops whose snapshot_time holds one remote DC's entry 2^33 us behind (a "
                         "partitioned DC): outside the packed view's window, read from the full columns")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the secondary lines (c3: cached c3, the indexed reads, c4, c5 and c2; single GPU "
                         "only)")
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

    cfg = dict(CONFIGS[args.config])
    if args.escape:
        cfg["escape"] = args.escape
        cfg["desc"] += f", {args.escape:.0%} of ops with a lagging-DC entry (escaped from the packed view)"
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

    def barrier():
        torch.cuda.synchronize()
        mat.sync()
        if pg is not None:
            pg.barrier()

    level = {"none": abi.AM_INDEX_NONE, "zones": abi.AM_INDEX_ZONES, "exact": abi.AM_INDEX_EXACT,
             "summaries": abi.AM_INDEX_SUMMARIES}[args.index]
    # ---- this GPU's op log, generated in HBM ----
    st = Step(mat, comm, cfg, rank, world, level)
    if args.base == "cached":
        st.populate()
    m = measure(st, args.base, args.steps, args.warmup, barrier, pg)
    if level == abi.AM_INDEX_NONE:
        assert m["skipped"] == 0 and m["rskip"] == 0, "the op-streaming headline skipped ops"

    n_dc, n_keys, type_ = cfg["n_dc"], cfg["n_keys"], cfg["type"]
    total_ops = world * st.n_ops * args.steps
    value = total_ops / m["dt"]
    workload = f"{args.config}: {cfg['desc']}"
    single = type_ in (abi.AM_PN, abi.AM_LWW)
    dt, kern_ms, achieved, logical = m["dt"], m["kern_ms"], m["achieved"], m["logical"]
    out = {
        "metric": "CRDT ops materialized/sec (whole node) + % HBM peak",
        "value": value,
        "unit": "ops/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "step_ms_hip_events": {"median": float(np.median(m["step_ev"])), "mean": float(np.mean(m["step_ev"])),
                               "min": float(np.min(m["step_ev"])), "n": len(m["step_ev"])},
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": f"synthetic (counter-based splitmix64 op logs generated in HBM; seed {hex(st.p.seed)})",
        "config": {"workload": workload, "keys_per_gpu": n_keys, "ops_per_gpu": st.n_ops, "n_dc": n_dc,
                   "snapshot_quantile": Q, "partitions": N_PARTITIONS, "parallelism": f"partition-sharded x{world}",
                   "key_placement": "rank r holds the keys with am_key_partition(key, 64) % N == r",
                   "step": "GST min all-reduce (RCCL) + materialize all keys" if args.base == "fresh" else
                           "GST min all-reduce (RCCL) + am_snapcache_read of all keys (read/6: cached base at "
                           "q=0.5, materialize/4, write-back); cache rebuilt between steps, untimed; HIP-event "
                           "timing of each step",
                   "base": args.base, "zone_index": INDEX_NAMES[level],
                   "store_build_s": st.build_s, "src_sha16": src_sha16()},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "model": "layout bytes (DESIGN.md 4): what the kernels stream of this build's HBM layout -- "
                              "commit vectors (packed: 4*D per op; lag view, for the reads of the tiers that stream it "
                              "(bench.lag_keys): 4 + 2*D per op and 4*D per read), "
                              "payload, 4 B per token-group record or 8 B per group-mask op, per-read metadata and "
                              "outputs; every op streamed (no zone index)"
                              if level == abi.AM_INDEX_NONE else
                              "layout bytes (DESIGN.md 4) minus the commit vectors / records the zone index stood in for",
                     "traffic": load_traffic(args.config if args.base == "fresh" else args.config + "_cached", workload,
                                             INDEX_NAMES[level]),
                     "kernel": ("am_snapcache_read (select + materialize tiers + store)" if args.base == "cached"
                                else "k_stream" if single else
                                "am_materialize (all tiers: k_stream, k_rows, k_grp_*, k_sets, k_big_*)"),
                     "kernel_ms": kern_ms,
                     "kernel_ms_median": m["kern_ms_median"],
                     "logical": {"model": "SURVEY.md 8(d) B_op / B_key (the reference's per-op record: "
                                          "8*D + 17 + P_type per op)", "bytes_per_launch": logical,
                                 "bytes_per_s": logical / (kern_ms * 1e-3),
                                 "frac_of_peak": logical / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS},
                     "alg_bytes_per_launch": m["alg_bytes"],
                     "ops_skipped_per_launch": m["skipped"], "records_skipped_per_launch": m["rskip"],
                     "gsum_words_per_launch": m["gsw"],
                     "layout": ("lag view (u32 commit time + u16 lag per DC, relative to per-key bases)"
                                if lag_split(cfg, st.dlog, level) else
                                "packed (u32 commit vectors relative to a per-key time base)")
                               + "; set effects as u32 token-group records" if m["packed"] else "full"},
        "cpu_baseline": None,
    }

    secondary = world == 1 and args.config == "c3" and args.base == "fresh" and not args.no_secondary
    if secondary:
        sec = {}
        ksteps = max(5, min(args.steps, 10))
        # read/6 steady state: the same store through the snapshot cache, every op streamed
        st.populate()
        mc = measure(st, "cached", ksteps, 2, barrier, pg)
        sec["c3_cached"] = summary(st, mc, world, "c3 --base cached: read/6 through the device snapshot cache "
                                                  "(q = 0.5 bases), materialize/4, write-back")
        sec["c3_cached"]["traffic"] = load_traffic("c3_cached", f"c3: {CONFIGS['c3']['desc']}", "none")
        # the zone index: its build cost, and what it buys a fresh and a cached read
        ims = st.reindex(abi.AM_INDEX_SUMMARIES)
        mi = measure(st, "fresh", ksteps, 2, barrier, pg)
        st.populate()
        mic = measure(st, "cached", ksteps, 2, barrier, pg)
        out["indexed"] = {"index_build_ms": ims, "zone_index": INDEX_NAMES[abi.AM_INDEX_SUMMARIES],
                          "note": "am_store_index rebuild (k_zone + k_zsum_size + scan + k_zsum_fill, wall clock); "
                                  "am_store_apply keeps it current in place (DESIGN.md 4b)",
                          "fresh": summary(st, mi, world, "c3 fresh, zone index on"),
                          "cached": summary(st, mic, world, "c3 cached, zone index on")}
        st.close()
        st = None
        # the north-star mix (BASELINE.json configs[3] per GPU)
        # the other BASELINE.json configs, each on its own store (C4: the north-star mix)
        for c in ("c4", "c5", "c2"):
            sx = Step(mat, comm, CONFIGS[c], rank, world, abi.AM_INDEX_NONE)
            mx = measure(sx, "fresh", ksteps, 2, barrier, pg)
            sec[c] = summary(sx, mx, world, f"{c}: " + CONFIGS[c]["desc"])
            sec[c]["traffic"] = load_traffic(c, f"{c}: " + CONFIGS[c]["desc"], "none")
            sx.close()
        out["secondary"] = sec
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        p = st.p if st is not None else synth_params(cfg, rank, world)
        out["cpu_baseline"] = cpu_baseline(cfg, p, budget_s=args.cpu_budget, cached=args.base == "cached")
    if rank == 0:
        print(json.dumps(out), flush=True)
    mat.L.am_comm_destroy(comm)
    if st is not None:
        st.close()
    mat.close()
    if pg is not None:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
