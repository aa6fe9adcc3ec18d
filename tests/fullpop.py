"""TEST INFRASTRUCTURE: full-population parity of a device-generated config.

Every read of one batch over every key of a synthetic store (bench.py's step: one
MinSnapshotTime, base ignore) is compared with the C oracle (oracle/am_oracle.c, the
restatement of clocksi_materializer:materialize/4, src/clocksi_materializer.erl:82-268) run
over the host-regenerated log (am_synth_host is bit-identical per key), in key chunks on a
thread pool.  The per-key output contract (src/clocksi_materializer.erl:89-101) is checked
column by column: status, NewLastOp, LastOpCt (clock, presence, ignore), IsNewSS, Count, the
flags, and the value (PN sum; LWW {Ts, Value} and the binary flag; AW / MV pairs in output
order; bounded-counter (slot, value) entries)."""
from __future__ import annotations

import ctypes
import os
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from antidote_amd import abi, synth
from oracle import amo

COMMON_COLS = ("new_last_op", "last_ct_pres", "last_ct_ignore", "is_new_ss", "count", "flags")
# value columns by type: PN v0; LWW v0, v1, vflag (AW / MV / bounded counter: the value CSR)
VALUE_COLS = {abi.AM_PN: ("v0",), abi.AM_LWW: ("v0", "v1", "vflag")}


def read_caps(kt: np.ndarray, n_dc: int, set_cap: int) -> np.ndarray:
    """Value room per read: every orddict entry of a bounded counter, set_cap pairs otherwise
    (devbatch.DeviceReads' rule)."""
    return np.where(kt == abi.AM_BCOUNTER, n_dc * n_dc + n_dc, set_cap).astype(np.uint64)


def oracle_chunk(p: abi.am_synth_params, k0: int, nk: int, clock, set_cap: int) -> dict:
    """The oracle's results for reads of keys [k0, k0 + nk) at the batch clock: result columns
    (numpy, read order) plus the value CSR (set_off relative to the chunk)."""
    log = synth.host_log(p, k0, nk)
    nd = p.n_dc
    kt = log.key_type[:nk].copy()
    key = np.arange(nk, dtype=np.uint64)
    rvc = np.asarray([int(c) for c in clock], np.uint64)
    rpres = np.asarray([(1 << nd) - 1], np.uint32)
    b = abi.am_read_batch()
    b.n_reads, b.per_read_clock, b.type_hint = nk, 0, 0
    b.key, b.type, b.read_vc, b.read_pres = key.ctypes.data, kt.ctypes.data, rvc.ctypes.data, rpres.ctypes.data
    n1 = max(nk, 1)
    out = {"status": np.full(n1, 99, np.int32), "new_last_op": np.zeros(n1, np.int64),
           "last_ct": np.zeros((nd, n1), np.uint64), "last_ct_pres": np.zeros(n1, np.uint32),
           "last_ct_ignore": np.zeros(n1, np.uint8), "is_new_ss": np.zeros(n1, np.uint8),
           "count": np.zeros(n1, np.uint32), "flags": np.zeros(n1, np.uint8), "v0": np.zeros(n1, np.int64),
           "v1": np.zeros(n1, np.uint64), "vflag": np.zeros(n1, np.uint8)}
    caps = read_caps(kt, nd, set_cap)
    so = np.zeros(nk + 1, np.uint64)
    so[1:] = np.cumsum(caps, dtype=np.uint64)
    tot = max(int(so[-1]), 1)
    out.update(set_off=so, set_len=np.zeros(n1, np.uint32), set_a=np.zeros(tot, np.uint64),
               set_b=np.zeros(tot, np.uint64))
    r = abi.am_read_result()
    for f in ("status", "new_last_op", "last_ct", "last_ct_pres", "last_ct_ignore", "is_new_ss", "count", "flags"):
        setattr(r, f, out[f].ctypes.data)
    r.value.v0, r.value.v1, r.value.vflag = out["v0"].ctypes.data, out["v1"].ctypes.data, out["vflag"].ctypes.data
    r.value.set_off, r.value.set_len = out["set_off"].ctypes.data, out["set_len"].ctypes.data
    r.value.set_a, r.value.set_b = out["set_a"].ctypes.data, out["set_b"].ctypes.data
    s = log.as_struct()
    amo.lib().amo_materialize_range(ctypes.byref(s), ctypes.byref(b), 0, nk, ctypes.byref(r))
    out["key_type"] = kt
    return out


def device_results(dr) -> dict:
    """Every result column of a DeviceReads batch, on the host."""
    h = dr.host()
    if dr.set_len is not None:
        h["set_off"] = dr.set_off.cpu().numpy().view(np.uint64)
        h["set_len"] = dr.set_len.cpu().numpy().view(np.uint32)
        h["set_a"] = dr.set_a.cpu().numpy().view(np.uint64)
        h["set_b"] = dr.set_b.cpu().numpy().view(np.uint64)
    return h


def _pair_index(off: np.ndarray, lens: np.ndarray) -> np.ndarray:
    """Flat indices of pairs j < lens[i] at off[i] + j, read by read."""
    lens = lens.astype(np.int64)
    tot = int(lens.sum())
    if tot == 0:
        return np.zeros(0, np.int64)
    starts = off.astype(np.int64)
    first = np.repeat(starts - (np.cumsum(lens) - lens), lens)
    return first + np.arange(tot, dtype=np.int64)


def compare_chunk(dev: dict, ref: dict, k0: int, nk: int) -> np.ndarray:
    """Chunk-relative indices of the reads whose outputs differ (any column)."""
    bad = np.zeros(nk, bool)
    st_ok = ref["status"][:nk] == 0
    bad |= dev["status"][k0:k0 + nk] != ref["status"][:nk]
    for c in COMMON_COLS:
        # outputs of failed reads are unspecified, only their status counts
        bad |= (dev[c][k0:k0 + nk] != ref[c][:nk]) & st_ok
    kt = ref["key_type"][:nk]
    for t, cols in VALUE_COLS.items():
        for c in cols:
            bad |= (dev[c][k0:k0 + nk] != ref[c][:nk]) & st_ok & (kt == t)
    pres = ref["last_ct_pres"][:nk].astype(np.int64)
    for d in range(ref["last_ct"].shape[0]):
        has = (((pres >> d) & 1) == 1) & (ref["last_ct_ignore"][:nk] == 0) & st_ok
        bad |= (dev["last_ct"][d, k0:k0 + nk] != ref["last_ct"][d, :nk]) & has
    if "set_len" in dev:
        csr = (kt == abi.AM_AWSET) | (kt == abi.AM_MVREG) | (kt == abi.AM_BCOUNTER)
        dl, rl = dev["set_len"][k0:k0 + nk], ref["set_len"][:nk]
        bad |= (dl != rl) & st_ok & csr
        same = (dl == rl) & st_ok & csr & (rl > 0)
        idx = np.nonzero(same)[0]
        if len(idx):
            lens = rl[idx]
            di = _pair_index(dev["set_off"][k0 + idx], lens)
            ri = _pair_index(ref["set_off"][idx], lens)
            diff = (dev["set_a"][di] != ref["set_a"][ri]) | (dev["set_b"][di] != ref["set_b"][ri])
            if diff.any():
                owner = np.repeat(idx, lens.astype(np.int64))
                bad[np.unique(owner[diff])] = True
    return np.nonzero(bad)[0]


def chunks(n_keys: int, lens: np.ndarray, max_ops: int = 1 << 22, max_keys: int = 1 << 16):
    """[k0, nk) key ranges of at most max_ops ops (a longer key alone) and max_keys keys."""
    out, k0 = [], 0
    cum = np.concatenate([[0], np.cumsum(lens.astype(np.int64))])
    while k0 < n_keys:
        k1 = int(np.searchsorted(cum, cum[k0] + max_ops, side="right")) - 1
        k1 = max(k0 + 1, min(k1, k0 + max_keys, n_keys))
        out.append((k0, k1 - k0))
        k0 = k1
    return out


def full_parity(p: abi.am_synth_params, clock, set_cap: int, dev: dict, lens: np.ndarray, workers: int = 0):
    """Compare every read of `dev` (device results over keys [0, n_keys)) with the oracle.
    Returns (reads checked, ops covered, mismatching key indices)."""
    workers = workers or max(1, min(16, os.cpu_count() or 1))
    parts = chunks(int(p.n_keys), lens)

    done = [0]
    lock = threading.Lock()

    def one(c):
        k0, nk = c
        ref = oracle_chunk(p, k0, nk, clock, set_cap)
        assert (ref["key_type"] == dev["_key_type"][k0:k0 + nk]).all(), "host regeneration differs (key types)"
        bad = k0 + compare_chunk(dev, ref, k0, nk)
        with lock:  # progress (a long check must not look hung)
            done[0] += 1
            if done[0] % max(1, len(parts) // 8) == 0:
                print(f"  full parity: {done[0]}/{len(parts)} chunks", flush=True)
        return bad

    with ThreadPoolExecutor(workers) as ex:
        bad = np.concatenate([np.zeros(0, np.int64)] + list(ex.map(one, parts)))
    return int(p.n_keys), int(lens.sum()), bad
