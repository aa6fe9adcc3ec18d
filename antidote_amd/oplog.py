"""Host-side encoding of the reference's ops cache into the HBM structure-of-arrays
layout of include/antidote_mat.h (am_op_log), read batches (am_read_batch) and
their decoding (am_read_result).

This is the ingestion side of materializer_vnode:op_insert_gc/3
(src/materializer_vnode.erl:622-647): one #clocksi_payload{} (include/antidote.hrl:197-204)
becomes one row of the op columns; ops of a key stay oldest -> newest, as in the
ETS tuple (slots FIRST_OP..FIRST_OP+Length-1, include/antidote.hrl:81-90).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import abi

U64 = np.uint64


@dataclass
class Op:
    """One committed effect (#clocksi_payload{}) with DCs already mapped to indices."""
    type: int
    commit_dc: int
    commit_time: int
    snap: Dict[int, int]                 # snapshot_time as {dc_index: time}
    effect: Any                          # see encode_effect
    txid: Optional[int] = None
    op_id: Optional[int] = None
    bad: bool = False                    # Type:update/2 raises on this effect


def encode_effect(type_: int, eff) -> Tuple[int, int, int, List[int]]:
    """-> (kind, p0, p1, var words).  Effect shapes (antidote_crdt downstream effects):
    PN int | LWW (ts, value) | MV ('assign', value, token, [overridden]) or ('reset', [overridden])
    | AWSET [(elem, [add_tokens], [remove_tokens]), ...] sorted by elem
    | BCOUNTER ('increment', V, id) | ('decrement', V, id) | ('transfer', V, to, from)."""
    if type_ == abi.AM_PN:
        return 0, int(eff) & 0xFFFFFFFFFFFFFFFF, 0, []
    if type_ == abi.AM_LWW:
        ts, val = eff
        return 0, int(ts), int(val), []
    if type_ == abi.AM_MVREG:
        if eff[0] == "reset":
            return 1, 0, 0, [int(t) for t in eff[1]]
        _, val, tok, ovr = eff
        return 0, int(val), int(tok), [int(t) for t in ovr]
    if type_ == abi.AM_AWSET:
        words: List[int] = []
        for elem, add, rm in eff:
            words += [int(elem), len(add), len(rm)] + [int(t) for t in add] + [int(t) for t in rm]
        return 0, 0, 0, words
    if type_ == abi.AM_BCOUNTER:
        kind = {"increment": 0, "decrement": 1, "transfer": 2}[eff[0]]
        if kind == 2:
            _, v, to, frm = eff
        else:
            _, v, frm = eff
            to = frm
        return kind, int(v) & 0xFFFFFFFFFFFFFFFF, int(frm) | (int(to) << 8), []
    raise ValueError(type_)


class HostLog:
    """SoA op log in host memory (numpy), the layout am_store_create uploads."""

    def __init__(self, n_dc: int, keys: Sequence[Sequence[Op]], key_types: Optional[Sequence[int]] = None,
                 key_id_base: Optional[Sequence[int]] = None, partial: Optional[bool] = None):
        if not 1 <= n_dc <= abi.AM_MAX_DC:
            raise ValueError("n_dc out of range")
        self.n_dc = n_dc
        n_keys = len(keys)
        lens = [len(k) for k in keys]
        n_ops = int(sum(lens))
        self.n_keys, self.n_ops = n_keys, n_ops
        self.key_off = np.zeros(n_keys + 1, U64)
        self.key_off[1:] = np.cumsum(lens, dtype=U64)
        self.key_type = np.zeros(max(n_keys, 1), np.uint8)
        self.key_flags = np.zeros(max(n_keys, 1), np.uint8)
        n_alloc = max(n_ops, 1)
        self.op_meta = np.zeros(n_alloc, np.uint8)
        self.commit_time = np.zeros(n_alloc, U64)
        self.snap_vc = np.zeros((n_dc, n_alloc), U64)
        self.snap_pres = np.zeros(n_alloc, np.uint32)
        self.p0 = np.zeros(n_alloc, U64)
        self.p1 = np.zeros(n_alloc, U64)
        self.var_off = np.zeros(n_ops + 1, U64)
        var: List[int] = []
        all_mask = (1 << n_dc) - 1
        need_pres = False
        has_txid = any(op.txid is not None for k in keys for op in k)
        has_opid = any(op.op_id is not None for k in keys for op in k)
        self.op_txid = np.zeros(n_alloc, U64) if has_txid else None
        self.op_id = np.zeros(n_alloc, U64) if has_opid else None
        self.key_id_base = np.asarray(key_id_base, U64) if key_id_base is not None else None
        q = 0
        for k, ops in enumerate(keys):
            types = {op.type for op in ops}
            if key_types is not None:
                self.key_type[k] = key_types[k]
            elif ops:
                self.key_type[k] = ops[0].type
            if len(types) > 1 or (key_types is not None and types and types != {key_types[k]}):
                self.key_flags[k] |= abi.AM_KEY_MIXED_TYPES
            for op in ops:
                kind, p0, p1, words = encode_effect(op.type, op.effect) if not op.bad else (0, 0, 0, [])
                self.op_meta[q] = abi.make_meta(op.commit_dc, kind, op.bad)
                self.commit_time[q] = op.commit_time
                pres = 0
                for d, t in op.snap.items():
                    self.snap_vc[d, q] = t
                    pres |= 1 << d
                self.snap_pres[q] = pres
                if pres != all_mask:
                    need_pres = True
                self.p0[q] = p0
                self.p1[q] = p1
                var += words
                self.var_off[q + 1] = len(var)
                if has_txid:
                    self.op_txid[q] = 0 if op.txid is None else op.txid
                if has_opid:
                    self.op_id[q] = op.op_id
                q += 1
        if partial is False:
            need_pres = False
        if not need_pres and partial is not True:
            self.snap_pres = None
        self.var_data = np.asarray(var if var else [0], U64)
        self.n_var = len(var)
        self.has_var = self.n_var > 0
        self._struct = None

    def as_struct(self) -> abi.am_op_log:
        s = abi.am_op_log()
        s.n_dc, s.n_keys, s.n_ops, s.n_var = self.n_dc, self.n_keys, self.n_ops, self.n_var
        s.snap_stride = self.snap_vc.shape[1]
        p = lambda a: None if a is None else a.ctypes.data  # noqa: E731
        s.key_off, s.key_id_base, s.key_type, s.key_flags = (p(self.key_off), p(self.key_id_base),
                                                             p(self.key_type), p(self.key_flags))
        s.op_meta, s.commit_time, s.snap_vc, s.snap_pres = (p(self.op_meta), p(self.commit_time),
                                                            p(self.snap_vc), p(self.snap_pres))
        s.op_txid, s.op_id, s.p0, s.p1 = p(self.op_txid), p(self.op_id), p(self.p0), p(self.p1)
        s.var_off = p(self.var_off) if self.has_var else None
        s.var_data = p(self.var_data) if self.has_var else None
        self._struct = s
        return s


@dataclass
class Read:
    """Inputs of one materialize/4 call for one key of the log."""
    key: int
    type: int
    clock: Dict[int, int]                        # MinSnapshotTime
    txid: Optional[int] = None                   # None = ignore
    base_clock: Optional[Dict[int, int]] = None  # None = ignore
    base_last_op: int = 0
    base_value: Any = None                       # None = Type:new()


def _pres(clock: Dict[int, int]) -> int:
    m = 0
    for d in clock:
        m |= 1 << d
    return m


def bc_pairs(value, n_dc: int) -> List[Tuple[int, int]]:
    """A bounded counter's ({(From, To): N}, {Id: N}) as the ABI's (slot, value) entries: P at
    From*n_dc+To, then D at n_dc*n_dc+Id, slot order (include/antidote_mat.h am_values)."""
    pdict, ddict = value
    out = [(f * n_dc + t, int(v)) for (f, t), v in pdict.items()] + [(n_dc * n_dc + d, int(v)) for d, v in ddict.items()]
    return [(s, int(np.array([v], np.int64).view(np.uint64)[0])) for s, v in sorted(out)]


def bc_dicts(pairs, n_dc: int):
    """The inverse of bc_pairs: (slot, value-bits) entries -> ({(From, To): N}, {Id: N})."""
    pd, dd = {}, {}
    for s, v in pairs:
        x = int(np.array([v], np.uint64).view(np.int64)[0])
        if s < n_dc * n_dc:
            pd[(s // n_dc, s % n_dc)] = x
        else:
            dd[s - n_dc * n_dc] = x
    return pd, dd


class HostBatch:
    """am_read_batch + am_read_result in host memory."""

    def __init__(self, n_dc: int, reads: Sequence[Read], set_capacity: Optional[Sequence[int]] = None):
        n = len(reads)
        self.n, self.n_dc, self.reads = n, n_dc, list(reads)
        self.key = np.asarray([r.key for r in reads] or [0], U64)
        self.type = np.asarray([r.type for r in reads] or [0], np.uint8)
        types = {r.type for r in reads}
        self.type_hint = types.pop() if len(types) == 1 else 0
        self.read_vc = np.zeros((n_dc, max(n, 1)), U64)
        self.read_pres = np.zeros(max(n, 1), np.uint32)
        self.txid = np.zeros(max(n, 1), U64)
        self.txid_valid = np.zeros(max(n, 1), np.uint8)
        self.base_ignore = np.ones(max(n, 1), np.uint8)
        self.base_vc = np.zeros((n_dc, max(n, 1)), U64)
        self.base_pres = np.zeros(max(n, 1), np.uint32)
        self.base_last_op = np.zeros(max(n, 1), np.int64)
        self.b_v0 = np.zeros(max(n, 1), np.int64)
        self.b_v1 = np.zeros(max(n, 1), U64)
        self.b_vflag = np.ones(max(n, 1), np.uint8)
        base_pairs: List[List[Tuple[int, int]]] = []
        for i, r in enumerate(reads):
            for d, t in r.clock.items():
                self.read_vc[d, i] = t
            self.read_pres[i] = _pres(r.clock)
            if r.txid is not None:
                self.txid[i] = r.txid
                self.txid_valid[i] = 1
            if r.base_clock is not None:
                self.base_ignore[i] = 0
                for d, t in r.base_clock.items():
                    self.base_vc[d, i] = t
                self.base_pres[i] = _pres(r.base_clock)
            self.base_last_op[i] = r.base_last_op
            pairs: List[Tuple[int, int]] = []
            bv = r.base_value
            if bv is not None:
                if r.type == abi.AM_PN:
                    self.b_v0[i] = bv
                elif r.type == abi.AM_LWW:
                    ts, val, isbin = bv
                    self.b_v0[i] = np.array([ts], np.uint64).view(np.int64)[0]
                    self.b_v1[i] = val
                    self.b_vflag[i] = 1 if isbin else 0
                elif r.type == abi.AM_AWSET:  # the orddict in state order (elems ascending)
                    pairs = [(int(a), int(b)) for a, b in bv]
                elif r.type == abi.AM_MVREG:  # a sorted list of {Value, Token}
                    pairs = sorted((int(a), int(b)) for a, b in bv)
                elif r.type == abi.AM_BCOUNTER:  # the P / D orddicts as (slot, value) entries
                    pairs = bc_pairs(bv, n_dc)
            base_pairs.append(pairs)
        self.has_txid = any(r.txid is not None for r in reads)
        self.has_base = any(r.base_clock is not None for r in reads)
        # base set CSR
        lens = [len(p) for p in base_pairs]
        self.b_set_off = np.zeros(n + 1, U64)
        self.b_set_off[1:] = np.cumsum(lens, dtype=U64) if n else []
        flat = [x for p in base_pairs for x in p]
        self.b_set_len = np.asarray(lens or [0], np.uint32)
        self.b_set_a = np.asarray([a for a, _ in flat] or [0], U64)
        self.b_set_b = np.asarray([b for _, b in flat] or [0], U64)
        # results
        self.status = np.full(max(n, 1), 99, np.int32)
        self.new_last_op = np.zeros(max(n, 1), np.int64)
        self.last_ct = np.zeros((n_dc, max(n, 1)), U64)
        self.last_ct_pres = np.zeros(max(n, 1), np.uint32)
        self.last_ct_ignore = np.zeros(max(n, 1), np.uint8)
        self.is_new_ss = np.zeros(max(n, 1), np.uint8)
        self.count = np.zeros(max(n, 1), np.uint32)
        self.flags = np.zeros(max(n, 1), np.uint8)
        self.v0 = np.zeros(max(n, 1), np.int64)
        self.v1 = np.zeros(max(n, 1), U64)
        self.vflag = np.zeros(max(n, 1), np.uint8)
        # default room per read: 64 set pairs; every orddict entry of a bounded counter
        caps = (list(set_capacity) if set_capacity is not None else
                [max(64, n_dc * n_dc + n_dc) if r.type == abi.AM_BCOUNTER else 64 for r in reads])
        self.o_set_off = np.zeros(n + 1, U64)
        self.o_set_off[1:] = np.cumsum(caps, dtype=U64) if n else []
        tot = int(self.o_set_off[-1]) if n else 0
        self.o_set_len = np.zeros(max(n, 1), np.uint32)
        self.o_set_a = np.zeros(max(tot, 1), U64)
        self.o_set_b = np.zeros(max(tot, 1), U64)

    def structs(self):
        p = lambda a: a.ctypes.data  # noqa: E731
        b = abi.am_read_batch()
        b.n_reads, b.per_read_clock, b.type_hint = self.n, 1, self.type_hint
        b.key, b.type, b.read_vc, b.read_pres = p(self.key), p(self.type), p(self.read_vc), p(self.read_pres)
        if self.has_txid:
            b.txid, b.txid_valid = p(self.txid), p(self.txid_valid)
        b.base_ignore = p(self.base_ignore)
        b.base_vc, b.base_pres, b.base_last_op = p(self.base_vc), p(self.base_pres), p(self.base_last_op)
        bv = b.base
        bv.v0, bv.v1, bv.vflag = p(self.b_v0), p(self.b_v1), p(self.b_vflag)
        bv.set_off, bv.set_len, bv.set_a, bv.set_b = (p(self.b_set_off), p(self.b_set_len), p(self.b_set_a),
                                                      p(self.b_set_b))
        r = abi.am_read_result()
        r.status, r.new_last_op, r.last_ct, r.last_ct_pres = (p(self.status), p(self.new_last_op), p(self.last_ct),
                                                              p(self.last_ct_pres))
        r.last_ct_ignore, r.is_new_ss, r.count, r.flags = (p(self.last_ct_ignore), p(self.is_new_ss),
                                                           p(self.count), p(self.flags))
        rv = r.value
        rv.v0, rv.v1, rv.vflag = p(self.v0), p(self.v1), p(self.vflag)
        rv.set_off, rv.set_len, rv.set_a, rv.set_b = (p(self.o_set_off), p(self.o_set_len), p(self.o_set_a),
                                                      p(self.o_set_b))
        self._keep = (b, r)
        return b, r

    # ---- decoding ----
    def value(self, i: int):
        t = self.reads[i].type
        if t == abi.AM_PN:
            return int(self.v0[i])
        if t == abi.AM_LWW:
            return (int(self.v0[i:i + 1].view(np.uint64)[0]), int(self.v1[i]), bool(self.vflag[i]))
        if t in (abi.AM_AWSET, abi.AM_MVREG):
            o, n = int(self.o_set_off[i]), int(self.o_set_len[i])
            return [(int(self.o_set_a[o + j]), int(self.o_set_b[o + j])) for j in range(n)]
        if t == abi.AM_BCOUNTER:
            o, n = int(self.o_set_off[i]), int(self.o_set_len[i])
            return bc_dicts([(int(self.o_set_a[o + j]), int(self.o_set_b[o + j])) for j in range(n)], self.n_dc)
        raise ValueError(t)

    def result(self, i: int):
        """('ok', Value, NewLastOp, LastOpCt, IsNewSS, Count, flags) or ('error', status)."""
        st = int(self.status[i])
        if st != 0:
            return ("error", st)
        ct = None if self.last_ct_ignore[i] else {d: int(self.last_ct[d, i]) for d in range(self.n_dc)
                                                   if (int(self.last_ct_pres[i]) >> d) & 1}
        return ("ok", self.value(i), int(self.new_last_op[i]), ct, bool(self.is_new_ss[i]), int(self.count[i]),
                int(self.flags[i]))
