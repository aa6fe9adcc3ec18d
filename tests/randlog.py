"""Random op logs for parity tests: the same log rendered three ways --
antidote_amd.oplog (the HBM SoA layout), and reference-shaped terms for the
Python restatement (oracle/ref_materializer.py)."""
import random
from typing import List

from antidote_amd import abi
from antidote_amd.oplog import Op, Read
from oracle import ref_materializer as R

TYPES = [abi.AM_PN, abi.AM_LWW, abi.AM_AWSET, abi.AM_MVREG, abi.AM_BCOUNTER]


def rand_effect(rng, t, n_dc, state):
    """A causally plausible effect; `state` carries per-key bookkeeping (live tokens)."""
    if t == abi.AM_PN:
        return rng.randint(-1000, 1000)
    if t == abi.AM_LWW:
        return (rng.choice([0, rng.randint(1, 60)]) if rng.random() < 0.1 else rng.randint(1, 60),
                rng.randint(0, 5))
    if t == abi.AM_AWSET:
        # adds observe-and-replace the live tokens (antidote_crdt's add), or -- as a
        # concurrent add would -- leave some live, so an element can hold several tokens
        # (token-list order is part of the state); some effects add two tokens at once
        ents = []
        for e in sorted(rng.sample(range(6), rng.randint(1, 2))):
            live = state.setdefault(e, [])
            if rng.random() < 0.65:
                toks = []
                for _ in range(1 if rng.random() < 0.85 else 2):
                    toks.append(state.get("next", 100) + 1)
                    state["next"] = toks[-1]
                r = rng.random()
                rm = list(live) if r < 0.6 else (live[: len(live) // 2] if r < 0.8 else [])
                state[e] = toks + [x for x in live if x not in rm]
                ents.append((e, toks, rm))
            else:
                rm = list(live) if rng.random() < 0.8 else [rng.randint(100, 130)]
                state[e] = []
                ents.append((e, [], rm))
        return ents
    if t == abi.AM_MVREG:
        live = state.setdefault("mv", [])
        if rng.random() < 0.1:
            state["mv"] = []
            return ("reset", list(live))
        tok = state["next"] = state.get("next", 500) + 1
        ovr = list(live) if rng.random() < 0.85 else live[: len(live) // 2]
        state["mv"] = [x for x in live if x not in ovr] + [tok]
        return ("assign", rng.randint(0, 4), tok, ovr)
    if t == abi.AM_BCOUNTER:
        k = rng.choice(["increment", "decrement", "transfer"])
        if k == "transfer":
            return (k, rng.randint(1, 50), rng.randrange(n_dc), rng.randrange(n_dc))
        return (k, rng.randint(1, 50), rng.randrange(n_dc))
    raise ValueError(t)


def rand_key_ops(rng, t, n_dc, n_ops, partial=False, txids=False, bad_rate=0.0, t0=None):
    ops = []
    state = {}
    clock = t0 if t0 is not None else 10
    for i in range(n_ops):
        clock += rng.randint(1, 4)
        dc = rng.randrange(n_dc)
        snap = {}
        for d in range(n_dc):
            if partial and d != dc and rng.random() < 0.25:
                continue
            snap[d] = max(0, clock - rng.randint(1, 12))
        if partial and rng.random() < 0.15:
            snap.pop(dc, None)
        ops.append(Op(type=t, commit_dc=dc, commit_time=clock, snap=snap, effect=rand_effect(rng, t, n_dc, state),
                      txid=rng.randint(1, 5) if txids else None, bad=rng.random() < bad_rate))
    return ops


def rand_clock(rng, n_dc, lo, hi, partial=False):
    c = {}
    for d in range(n_dc):
        if partial and rng.random() < 0.2:
            continue
        c[d] = rng.randint(lo, hi)
    return c


# ---------------------------------------------------------------- reference terms
def effect_term(t, eff):
    if t == abi.AM_PN:
        return eff
    if t == abi.AM_LWW:
        return tuple(eff)
    if t == abi.AM_AWSET:
        return [(e, list(a), list(r)) for e, a, r in eff]
    if t == abi.AM_MVREG:
        if eff[0] == "reset":
            return ("reset", list(eff[1]))
        return (eff[1], eff[2], list(eff[3]))
    if t == abi.AM_BCOUNTER:
        if eff[0] == "transfer":
            return (("transfer", eff[1], eff[2]), eff[3])
        return ((eff[0], eff[1]), eff[2])
    raise ValueError(t)


def payload_term(op: Op, key="k"):
    eff = ("bad_effect", "x") if op.bad else effect_term(op.type, op.effect)
    snap = dict(op.snap)
    return R.Payload(key=key, type=op.type, op_param=eff, snapshot_time=snap,
                     commit_time=(op.commit_dc, op.commit_time), txid=op.txid if op.txid is not None else ("no", 0))


def base_state_term(t, v):
    """Base value in our encoding -> reference state."""
    if v is None:
        return R.crdt_new(t)
    if t == abi.AM_PN:
        return v
    if t == abi.AM_LWW:
        ts, val, isbin = v
        return (ts, R.Bin(b"") if isbin else val)
    if t == abi.AM_AWSET:  # ordered (elem, token) pairs: elems ascending, token lists in state order
        d = {}
        for e, tok in v:
            d.setdefault(e, []).append(tok)
        return sorted(d.items(), key=lambda kv: kv[0])
    if t == abi.AM_MVREG:
        return sorted(v)
    if t == abi.AM_BCOUNTER:
        p, dd = v
        return (sorted(p.items()), sorted(dd.items()))
    raise ValueError(t)


def canon_state(t, s):
    """Reference state -> the canonical rendering the ABI returns."""
    if t == abi.AM_PN:
        return s
    if t == abi.AM_LWW:
        ts, val = s
        return (ts, 0, True) if isinstance(val, bytes) else (ts, val, False)
    if t == abi.AM_AWSET:  # the orddict flattened in order: token lists are compared as ordered lists
        return [(e, tok) for e, toks in s for tok in toks]
    if t == abi.AM_MVREG:
        return sorted(set(s))
    if t == abi.AM_BCOUNTER:
        p, d = s
        return (dict(p), dict(d))
    raise ValueError(t)


def ref_materialize(t, ops: List[Op], read: Read):
    """Run the Python restatement on one key; returns the ABI-shaped result tuple."""
    ops_newest = [(i + 1 if op.op_id is None else op.op_id, payload_term(op)) for i, op in enumerate(ops)][::-1]
    base_ct = R.IGNORE if read.base_clock is None else dict(read.base_clock)
    resp = R.SnapshotGetResponse(ops_list=ops_newest, number_of_ops=len(ops),
                                 materialized_snapshot=R.MatSnapshot(read.base_last_op,
                                                                     base_state_term(t, read.base_value)),
                                 snapshot_time=base_ct, is_newest_snapshot=True)
    R.MissingDcLog.count = 0
    try:
        r = R.materialize(read.type, R.IGNORE if read.txid is None else read.txid, dict(read.clock), resp)
    except R.CorruptedOpsCache:
        return ("error", abi.AM_ERR_CORRUPTED_OPS_CACHE)
    if r[0] == "error":
        return ("error", abi.AM_ERR_UNEXPECTED_OPERATION)
    _, val, nlo, ct, newss, count = r
    flags = abi.AM_FLAG_MISSING_DC_LOGGED if R.MissingDcLog.count else 0
    return ("ok", canon_state(read.type, val), nlo, None if ct == R.IGNORE else dict(ct), newss, count, flags)


def caps_for(reads, n_dc, cap):
    """Result room per read: `cap` set pairs, and every orddict entry of a bounded counter
    (n_dc^2 + n_dc (slot, value) entries; include/antidote_mat.h am_values)."""
    return [max(cap, n_dc * n_dc + n_dc) if r.type == abi.AM_BCOUNTER else cap for r in reads]
