"""TEST INFRASTRUCTURE ONLY -- never imported by the product path.

Pure-Python, line-by-line restatement of the AntidoteDB snapshot-read hot path,
used as the *parity oracle* for small cases (the EUnit known-answer tests and
the vnode-level cache/GC tests).  The fast C restatement (``oracle/am_oracle.c``)
is cross-checked against this module on random logs.

Restated reference functions (paths relative to /root/reference):
  * vectorclock (hex ``vectorclock`` 0.1.0, rebar.lock:44, NOT vendored): dict
    based clocks; ``le`` over the union of keys with a missing entry read as 0.
  * materializer:belongs_to_snapshot_op/3          src/materializer.erl:102-106
  * materializer:update_snapshot/3                 src/materializer.erl:52-58
  * materializer:materialize_eager/3               src/materializer.erl:62-70
  * clocksi_materializer:get_first_id/1            src/clocksi_materializer.erl:51-63
  * clocksi_materializer:materialize/4             src/clocksi_materializer.erl:89-101
  * clocksi_materializer:apply_operations/4        src/clocksi_materializer.erl:113-121
  * clocksi_materializer:materialize_intern/11     src/clocksi_materializer.erl:157-171
  * clocksi_materializer:materialize_intern_perform/12  :173-197
  * clocksi_materializer:is_op_in_snapshot/7       src/clocksi_materializer.erl:216-268
  * vector_orddict (get_smaller, insert, insert_bigger, sublist, first, last,
    filter, is_concurrent_with_any)                src/vector_orddict.erl:42-183
  * materializer_vnode internal_read / get_from_snapshot_cache /
    materialize_snapshot / internal_store_ss / snapshot_insert_gc / prune_ops /
    check_filter / op_insert_gc                    src/materializer_vnode.erl:342-647
  * stable_time_functions:get_min_time/1, update_func_min/2
                                                   src/stable_time_functions.erl:42-85
  * meta_data_sender:update_stable/3               src/meta_data_sender.erl:342-356
  * dc_utilities:get_stable_snapshot/0 (gr mode)   src/dc_utilities.erl:246-279
  * log_utilities:convert_key/1, get_key_partition src/log_utilities.erl:60-118

The CRDT ``update/2`` functions live in the un-vendored dependency
``antidote_crdt`` (git SmallEndian/antidote_crdt @ 4157110c, rebar.lock:3-5).
``antidote_crdt_counter_pn`` is pinned by the reference's own EUnit KATs.  The
LWW register, add-wins set, MV register and bounded counter rules below are
restated from the published antidote_crdt algorithms and pinned only by the
state/effect *shapes* the reference's system tests assert
(test/singledc/object_log_state_SUITE.erl:96-105,
test/singledc/clocksi_SUITE.erl:160-205): **parity unpinned** at the numeric
level for those four types.
"""
from __future__ import annotations

from dataclasses import dataclass, field, replace
from typing import Any, Callable, Dict, List, Optional, Tuple

IGNORE = "ignore"          # the atom 'ignore'
UNDEFINED = "undefined"    # the atom 'undefined'

# type atoms -> small ints shared with the C ABI (include/antidote_mat.h)
PN, LWW, AWSET, MVREG, BCOUNTER = 1, 2, 3, 4, 5
TYPE_NAMES = {
    PN: "antidote_crdt_counter_pn",
    LWW: "antidote_crdt_register_lww",
    AWSET: "antidote_crdt_set_aw",
    MVREG: "antidote_crdt_register_mv",
    BCOUNTER: "antidote_crdt_counter_b",
}

FIRST_OP = 4              # include/antidote.hrl:90
SNAPSHOT_THRESHOLD = 10   # src/materializer_vnode.erl:37
SNAPSHOT_MIN = 3          # :39
OPS_THRESHOLD = 50        # :41
RESIZE_THRESHOLD = 5      # :44
MIN_OP_STORE_SS = 5       # :47


class CorruptedOpsCache(Exception):
    """erlang:error(corrupted_ops_cache), src/clocksi_materializer.erl:190-191."""


class UpdateError(Exception):
    pass


# ---------------------------------------------------------------------------
# Erlang term order (only the parts the CRDT values use: numbers < tuples < lists
# < binaries).  Used by the LWW max and the orddict/insert_sorted orderings.
# ---------------------------------------------------------------------------
class Bin(bytes):
    """An Erlang binary (sorts after every number, tuple and list)."""


def _rank(t):
    if isinstance(t, bool):
        raise TypeError("booleans are atoms; not used")
    if isinstance(t, int):
        return 0
    if isinstance(t, str):      # atoms
        return 1
    if isinstance(t, tuple):
        return 6
    if isinstance(t, list):
        return 8
    if isinstance(t, (bytes, Bin)):
        return 9
    raise TypeError(type(t))


def erl_cmp(a, b) -> int:
    ra, rb = _rank(a), _rank(b)
    if ra != rb:
        return -1 if ra < rb else 1
    if ra == 0 or ra == 1 or ra == 9:
        return (a > b) - (a < b)
    if ra == 6:  # tuples: size first, then elements
        if len(a) != len(b):
            return -1 if len(a) < len(b) else 1
        for x, y in zip(a, b):
            c = erl_cmp(x, y)
            if c:
                return c
        return 0
    # lists: lexicographic
    for x, y in zip(a, b):
        c = erl_cmp(x, y)
        if c:
            return c
    return (len(a) > len(b)) - (len(a) < len(b))


def erl_max(a, b):
    """erlang:max/2 -- the first argument wins a tie."""
    return b if erl_cmp(b, a) > 0 else a


# ---------------------------------------------------------------------------
# vectorclock (dict based).  keys are DC ids, values non-negative integers.
# ---------------------------------------------------------------------------
def vc_get(vc: dict, dc) -> int:
    return vc.get(dc, 0)


def vc_le(v1: dict, v2: dict) -> bool:
    """vectorclock:le/2: for every DC in keys(V1) ++ keys(V2), V1[dc] =< V2[dc] (missing = 0)."""
    for dc in list(v1.keys()) + list(v2.keys()):
        if not vc_get(v1, dc) <= vc_get(v2, dc):
            return False
    return True


def vc_eq(v1: dict, v2: dict) -> bool:
    return all(vc_get(v1, d) == vc_get(v2, d) for d in list(v1) + list(v2))


def vc_lt(v1, v2):
    return vc_le(v1, v2) and not vc_eq(v1, v2)


def vc_gt(v1, v2):
    """vectorclock:gt/2 = lt(V2, V1) (pinned by src/vector_orddict.erl:236-254: gt({dc1:0,dc2:3},{}) is true)."""
    return vc_lt(v2, v1)


def vc_conc(v1, v2):
    return not vc_le(v1, v2) and not vc_le(v2, v1)


def vc_all_dots_greater(v1, v2):
    """every entry of V1 strictly greater than V2's (missing = 0)."""
    return all(vc_get(v1, d) > vc_get(v2, d) for d in list(v1) + list(v2))


def vc_min2(v1: dict, v2: dict) -> dict:
    """vectorclock:min([V1, V2]): V2 with every DC of V1 lowered to min(V1[dc], V2[dc]), a DC
    missing from V2 read as 0 (a DC only in V2 keeps V2's entry).

    Pinned by the reference's own suites, not by a KAT: with dict:merge semantics (a DC missing
    from one clock keeps the other's entry) the first GC read of a key that was never read
    before -- op_insert_gc/3's read at NewId rem 50 == 0 (src/materializer_vnode.erl:633-640),
    whose dict then holds the new snapshot and the initial {} one (:394-397) -- gets a prune
    threshold equal to the new snapshot's clock, prunes every op, and prune_ops/2 leaves
    element(FIRST_OP+Len) = 0 as an op (:580-583), on which the next materialize/4 walk fails
    (src/clocksi_materializer.erl:173).  test/multidc/multiple_dcs_SUITE.erl:243-266 replicates
    100 adds to a key no one reads before op 99 and passes, so min({}, X) must not be X: with a
    missing DC read as 0 the threshold is all-zero while {} is kept and nothing is pruned."""
    out = dict(v2)
    for d, a in v1.items():
        b = v2.get(d, 0)
        out[d] = a if a < b else b
    return out


def vc_min(vcs):
    """vectorclock:min/1: min([V]) = V, min([V1, V2 | T]) = min([min2(V1, V2) | T])."""
    if not vcs:
        return {}
    acc = dict(vcs[0])
    for v in vcs[1:]:
        acc = vc_min2(acc, v)
    return acc


def gc_threshold(pruned) -> dict:
    """snapshot_insert_gc/4's prune threshold (src/materializer_vnode.erl:523-527):
    {CT, _} = vector_orddict:last(Pruned), then foldl over the entries (newest first) of
    Acc = vectorclock:min([CT1, Acc])."""
    ct, _s = vo_last(pruned)
    acc = ct
    for ct1, _st in pruned[0]:
        acc = vc_min([ct1, acc])
    return acc


# ---------------------------------------------------------------------------
# CRDT update/2 restatements (antidote_crdt, un-vendored)
# ---------------------------------------------------------------------------
def crdt_new(type_: int):
    if type_ == PN:
        return 0
    if type_ == LWW:
        return (0, Bin(b""))
    if type_ == AWSET:
        return []
    if type_ == MVREG:
        return []
    if type_ == BCOUNTER:
        return ([], [])
    raise ValueError(type_)


def _orddict_update_counter(d: list, key, incr: int) -> list:
    out = []
    done = False
    for k, v in d:
        if not done and erl_cmp(k, key) == 0:
            out.append((k, v + incr))
            done = True
        elif not done and erl_cmp(key, k) < 0:
            out.append((key, incr))
            out.append((k, v))
            done = True
        else:
            out.append((k, v))
    if not done:
        out.append((key, incr))
    return out


def erl_subtract(a: list, b: list) -> list:
    """Erlang's A -- B (lists:subtract/2): for each element of B, the first
    occurrence in A (if any) is removed; order of A is kept."""
    out = list(a)
    for x in b:
        for i, y in enumerate(out):
            if erl_cmp(x, y) == 0:
                del out[i]
                break
    return out


def _aw_apply_downstreams(ops: list, set_: list) -> list:
    # antidote_crdt_set_aw: merge of the (Elem-sorted) effect entries into the
    # Elem-sorted orddict; an element whose token list becomes empty is dropped.
    # Token lists keep the reference's list order: ToAdd ++ (Current -- ToRemove),
    # i.e. the newest add first.
    if not ops:
        return list(set_)
    if not set_:
        return [(e, list(add)) for (e, add, _rm) in ops if add]
    (e1, add, rm), ops_rest = ops[0], ops[1:]
    (e2, cur), set_rest = set_[0], set_[1:]
    c = erl_cmp(e1, e2)
    if c == 0:
        toks = list(add) + erl_subtract(cur, rm)
        tail = _aw_apply_downstreams(ops_rest, set_rest)
        return ([(e1, toks)] if toks else []) + tail
    if c > 0:
        return [(e2, cur)] + _aw_apply_downstreams(ops, set_rest)
    return ([(e1, list(add))] if add else []) + _aw_apply_downstreams(ops_rest, set_)


def _mv_insert_sorted(a, lst):
    for i, x in enumerate(lst):
        c = erl_cmp(a, x)
        if c < 0:
            return lst[:i] + [a] + lst[i:]
        if c == 0:
            return lst
    return lst + [a]


def crdt_update(type_: int, effect, state):
    """Type:update(Effect, State) -> {ok, NewState}; raises on a bad effect."""
    if type_ == PN:
        if not isinstance(effect, int) or isinstance(effect, bool):
            raise UpdateError(effect)
        return state + effect
    if type_ == LWW:
        if not (isinstance(effect, tuple) and len(effect) == 2 and isinstance(effect[0], int)):
            raise UpdateError(effect)
        return erl_max(effect, state)
    if type_ == AWSET:
        if not isinstance(effect, list):
            raise UpdateError(effect)
        return _aw_apply_downstreams(effect, state)
    if type_ == MVREG:
        if isinstance(effect, tuple) and len(effect) == 2 and effect[0] == "reset":
            ovr = effect[1]
            return [(v, t) for (v, t) in state if t not in ovr]
        if not (isinstance(effect, tuple) and len(effect) == 3):
            raise UpdateError(effect)
        val, tok, ovr = effect
        kept = [(v, t) for (v, t) in state if t not in ovr]
        return _mv_insert_sorted((val, tok), kept)
    if type_ == BCOUNTER:
        p, d = state
        if isinstance(effect, tuple) and len(effect) == 2 and isinstance(effect[0], tuple):
            (kind, *args), ident = effect[0], effect[1]
            if kind == "increment" and len(args) == 1:
                return (_orddict_update_counter(p, (ident, ident), args[0]), d)
            if kind == "decrement" and len(args) == 1:
                return (p, _orddict_update_counter(d, ident, args[0]))
            if kind == "transfer" and len(args) == 2:
                return (_orddict_update_counter(p, (ident, args[1]), args[0]), d)
        raise UpdateError(effect)
    raise UpdateError(effect)


def crdt_value(type_: int, state):
    if type_ == PN:
        return state
    if type_ == LWW:
        return state[1]
    if type_ == AWSET:
        return [e for e, _ in state]
    if type_ == MVREG:
        return [v for v, _ in state]
    if type_ == BCOUNTER:
        p, d = state
        return sum(v for (f, t), v in p if f == t) - sum(v for _, v in d)
    raise ValueError(type_)


def update_snapshot(type_, snapshot, op):
    """materializer:update_snapshot/3 (src/materializer.erl:52-58)."""
    try:
        return ("ok", crdt_update(type_, op, snapshot))
    except Exception:
        return ("error", ("unexpected_operation", op, TYPE_NAMES.get(type_, type_)))


def materialize_eager(type_, snapshot, effects):
    """materializer:materialize_eager/3 (src/materializer.erl:62-70)."""
    for eff in effects:
        st, res = update_snapshot(type_, snapshot, eff)
        if st == "error":
            return ("error", res)
        snapshot = res
    return snapshot


# ---------------------------------------------------------------------------
# clocksi_materializer
# ---------------------------------------------------------------------------
@dataclass
class Payload:
    """#clocksi_payload{} (include/antidote.hrl:197-204)."""
    key: Any
    type: int
    op_param: Any
    snapshot_time: dict
    commit_time: Tuple[Any, int]
    txid: Any


@dataclass
class MatSnapshot:
    """#materialized_snapshot{} (include/antidote.hrl:169-176)."""
    last_op_id: int
    value: Any


@dataclass
class SnapshotGetResponse:
    """#snapshot_get_response{} (include/antidote.hrl:255-266)."""
    ops_list: Any                   # list newest-first [(id, Payload)] or OpsTuple
    number_of_ops: int
    materialized_snapshot: MatSnapshot
    snapshot_time: Any              # dict or IGNORE
    is_newest_snapshot: bool


class OpsTuple:
    """The ETS ops-cache tuple {Key, {Length, ListLen}, OpCounter, Op_1..Op_Length, 0-pad}
    (include/antidote.hrl:81-90).  Element indices are Erlang 1-based."""

    def __init__(self, key, length, list_len, op_counter, ops):
        self.elems = [key, (length, list_len), op_counter] + list(ops)
        # erlang:make_tuple(FIRST_OP + ListLen, 0, ...): ListLen + 1 op slots
        self.elems += [0] * (FIRST_OP + list_len - len(self.elems))

    def element(self, i):
        return self.elems[i - 1]

    def copy(self):
        t = OpsTuple.__new__(OpsTuple)
        t.elems = list(self.elems)
        return t


class MissingDcLog:
    """Collects the logger:error calls of is_op_in_snapshot (src/clocksi_materializer.erl:246)."""
    count = 0


def belongs_to_snapshot_op(ss_time, op_dc_ct, op_ss) -> bool:
    """src/materializer.erl:102-106."""
    if ss_time == IGNORE:
        return True
    op_dc, op_ct = op_dc_ct
    op_ss1 = dict(op_ss)
    op_ss1[op_dc] = op_ct
    return not vc_le(op_ss1, ss_time)


def get_first_id(ops) -> int:
    """src/clocksi_materializer.erl:51-63."""
    if isinstance(ops, list):
        return 0 if not ops else ops[0][0]
    length, _ = ops.element(2)
    if length == 0:
        return 0
    return ops.element(FIRST_OP + length - 1)[0]


def is_op_in_snapshot(txid, op: Payload, op_dc_ct, op_ss, snapshot_time, last_snapshot, prev_time):
    """src/clocksi_materializer.erl:216-268 -> (include, already_in_prev, time)."""
    if belongs_to_snapshot_op(last_snapshot, op_dc_ct, op_ss) or (txid == op.txid):
        op_dc, op_ct = op_dc_ct
        op_ss_commit = dict(op_ss)
        op_ss_commit[op_dc] = op_ct
        prev_time2 = op_ss_commit if prev_time == IGNORE else prev_time
        acc, new_time = True, dict(prev_time2)
        for dc_op, time_op in op_ss_commit.items():
            if dc_op in snapshot_time:
                res1 = False if snapshot_time[dc_op] < time_op else acc
            else:
                MissingDcLog.count += 1
                res1 = False
            if dc_op in new_time:
                new_time[dc_op] = time_op if time_op > new_time[dc_op] else new_time[dc_op]
            else:
                new_time[dc_op] = time_op
            acc = res1
        if acc:
            return (True, False, new_time)
        return (False, False, prev_time)
    return (False, True, prev_time)


def materialize_intern(type_, op_list, last_op, first_hole, ss_commit_time, min_ss_time,
                       ops, txid, last_op_ct, new_ss, location):
    """src/clocksi_materializer.erl:157-197 (iterative form of the tail recursion)."""
    if isinstance(ops, list):
        seq = list(ops)                        # newest first
    else:
        length, _ = ops.element(2)
        seq = [ops.element(FIRST_OP + length - 1 - loc) for loc in range(location, length)]
    for op_id, op in seq:
        if type_ != op.type:
            raise CorruptedOpsCache()
        inc, in_prev, new_op_ct = is_op_in_snapshot(txid, op, op.commit_time, op.snapshot_time,
                                                    min_ss_time, ss_commit_time, last_op_ct)
        if inc:
            op_list = [op] + op_list
            last_op_ct = new_op_ct
            new_ss = True
        elif not in_prev:
            first_hole = op_id - 1
    return ("ok", op_list, first_hole, last_op_ct, new_ss)


def apply_operations(type_, snapshot, count, op_list):
    """src/clocksi_materializer.erl:113-121."""
    for op in op_list:
        st, res = update_snapshot(type_, snapshot, op.op_param)
        if st == "error":
            return ("error", res)
        snapshot = res
        count += 1
    return ("ok", snapshot, count)


def materialize(type_, txid, min_snapshot_time, resp: SnapshotGetResponse):
    """clocksi_materializer:materialize/4 (src/clocksi_materializer.erl:89-101).
    Returns ("ok", Value, NewLastOp, LastOpCt, IsNewSS, Count) or ("error", Reason)."""
    ss_ct = resp.snapshot_time
    ops = resp.ops_list
    last_op = resp.materialized_snapshot.last_op_id
    snapshot = resp.materialized_snapshot.value
    first_id = get_first_id(ops)
    _, op_list, new_last_op, last_op_ct, is_new_ss = materialize_intern(
        type_, [], last_op, first_id, ss_ct, min_snapshot_time, ops, txid, ss_ct, False, 0)
    r = apply_operations(type_, snapshot, 0, op_list)
    if r[0] == "ok":
        return ("ok", r[1], new_last_op, last_op_ct, is_new_ss, r[2])
    return r


# ---------------------------------------------------------------------------
# vector_orddict (src/vector_orddict.erl)
# ---------------------------------------------------------------------------
def vo_new():
    return ([], 0)


def vo_get_smaller(vector, vo):
    lst, _ = vo
    is_first = True
    for clock, val in lst:
        if vc_le(clock, vector):
            return ((clock, val), is_first)
        is_first = False
    return (UNDEFINED, is_first)


def vo_get_smaller_from_id(ident, time, vo):
    lst, size = vo
    if size == 0:
        return UNDEFINED
    for clock, val in lst:
        if vc_get(clock, ident) <= time:
            return (clock, val)
    return UNDEFINED


def vo_insert(vector, val, vo):
    lst, size = vo
    for i, (clock, _v) in enumerate(lst):
        if vc_all_dots_greater(vector, clock):
            return (lst[:i] + [(vector, val)] + lst[i:], size + 1)
    return (lst + [(vector, val)], size + 1)


def vo_insert_bigger(vector, val, vo):
    lst, size = vo
    if not lst and size == 0:
        return ([(vector, val)], 1)
    first_clock = lst[0][0]
    if not vc_le(vector, first_clock):
        return ([(vector, val)] + lst, size + 1)
    return (lst, size)


def vo_sublist(vo, start, length):
    res = vo[0][start - 1:start - 1 + length]
    return (res, len(res))


def vo_first(vo):
    return vo[0][0]


def vo_last(vo):
    return vo[0][-1]


def vo_filter(fun, vo):
    res = [e for e in vo[0] if fun(e)]
    return (res, len(res))


def vo_is_concurrent_with_any(vo, other):
    return any(vc_conc(c, other) for c, _ in vo[0])


# ---------------------------------------------------------------------------
# materializer_vnode caches (ETS replaced by dicts), src/materializer_vnode.erl
# ---------------------------------------------------------------------------
@dataclass
class VnodeState:
    ops_cache: Dict[Any, OpsTuple] = field(default_factory=dict)
    snapshot_cache: Dict[Any, Any] = field(default_factory=dict)


def internal_store_ss(key, snapshot: MatSnapshot, commit_time, should_gc, st: VnodeState):
    """:342-364."""
    sdict = st.snapshot_cache.get(key, vo_new())
    if sdict[1] > 0:
        _v, old = vo_first(sdict)
        should_insert = (snapshot.last_op_id - old.last_op_id) >= MIN_OP_STORE_SS
    else:
        should_insert = True
    if should_insert or should_gc:
        sdict1 = vo_insert_bigger(commit_time, snapshot, sdict)
        return snapshot_insert_gc(key, sdict1, should_gc, st)
    return False


def store_snapshot(txid, key, snapshot, time, should_gc, st):
    """:418-434 (the async store_ss command is applied synchronously here)."""
    internal_store_ss(key, snapshot, time, should_gc, st)


def fetch_updates_from_cache(st: VnodeState, key):
    """:456-464."""
    t = st.ops_cache.get(key)
    if t is None:
        return ([], 0)
    length, _ = t.element(2)
    return (t.copy(), length)


def update_snapshot_from_cache(resp, key, st):
    """:440-449."""
    (ss_ct, latest), is_first = resp
    ops, ops_len = fetch_updates_from_cache(st, key)
    return SnapshotGetResponse(ops_list=ops, number_of_ops=ops_len, is_newest_snapshot=is_first,
                               snapshot_time=ss_ct, materialized_snapshot=latest)


class LogColdPath(Exception):
    """get_from_snapshot_log -> logging_vnode:get_up_to_time (not part of the hot path)."""


def get_from_snapshot_cache(txid, key, type_, min_ss_time, st):
    """:384-413."""
    if key not in st.snapshot_cache:
        empty = MatSnapshot(last_op_id=0, value=crdt_new(type_))
        store_snapshot(txid, key, empty, {}, False, st)
        return update_snapshot_from_cache(((IGNORE, empty), True), key, st)
    found = vo_get_smaller(min_ss_time, st.snapshot_cache[key])
    if found[0] == UNDEFINED:
        raise LogColdPath(key)
    return update_snapshot_from_cache(found, key, st)


def materialize_snapshot(txid, key, type_, ss_time, should_gc, st, resp: SnapshotGetResponse):
    """:469-509."""
    if resp.number_of_ops == 0:
        return ("ok", resp.materialized_snapshot.value)
    r = materialize(type_, txid, ss_time, resp)
    if r[0] == "error":
        return r
    _, value, new_last_op, commit_time, was_updated, ops_added = r
    if commit_time == IGNORE:
        return ("ok", value)
    should_refresh = was_updated and resp.is_newest_snapshot and ops_added >= MIN_OP_STORE_SS
    if should_refresh or should_gc:
        store_snapshot(txid, key, MatSnapshot(new_last_op, value), commit_time, should_gc, st)
    return ("ok", value)


def internal_read(key, type_, min_ss_time, txid, should_gc, st):
    """:371-376."""
    resp = get_from_snapshot_cache(txid, key, type_, min_ss_time, st)
    return materialize_snapshot(txid, key, type_, min_ss_time, should_gc, st, resp)


def snapshot_insert_gc(key, sdict, should_gc, st: VnodeState):
    """:515-563."""
    if sdict[1] >= SNAPSHOT_THRESHOLD or should_gc:
        pruned = vo_sublist(sdict, 1, SNAPSHOT_MIN)
        commit_time = gc_threshold(pruned)
        t = st.ops_cache.get(key)
        if t is None:
            length, op_id, list_len, tup = 0, 0, 0, None
        else:
            length, list_len = t.element(2)
            op_id = t.element(3)
            tup = t
        new_length, pruned_ops = prune_ops(length, tup, commit_time)
        st.snapshot_cache[key] = pruned
        if new_length > list_len - RESIZE_THRESHOLD:
            new_list_len = list_len * 2
        else:
            half = list_len // 2
            if half <= OPS_THRESHOLD:
                new_list_len = list_len
            elif half - RESIZE_THRESHOLD > new_length:
                new_list_len = half
            else:
                new_list_len = list_len
        # erlang:make_tuple(FIRST_OP+NewListLen, 0, [{1,Key},{2,{NewLength,NewListLen}},{3,OpId}|PrunedOps])
        elems = [0] * (FIRST_OP + new_list_len)
        inits = [(1, key), (2, (new_length, new_list_len)), (3, op_id)] + pruned_ops
        for pos, v in inits:
            if pos - 1 >= len(elems):
                raise IndexError("make_tuple badarg")
            elems[pos - 1] = v
        nt = OpsTuple.__new__(OpsTuple)
        nt.elems = elems
        st.ops_cache[key] = nt
        return True
    st.snapshot_cache[key] = sdict
    return True


def prune_ops(length, tup, threshold):
    """:566-604 (check_filter inlined).  Keeps the quirk of element(FIRST_OP+Len) when all are pruned."""
    new_ops = []
    new_size = 0
    new_id = FIRST_OP
    for i in range(FIRST_OP, FIRST_OP + length):
        op = tup.element(i)
        _op_id, payload = op
        if belongs_to_snapshot_op(threshold, payload.commit_time, payload.snapshot_time):
            new_ops = [(new_id, op)] + new_ops
            new_id += 1
            new_size += 1
    if new_size == 0:
        if tup is None:   # element(FIRST_OP, {}) -> badarg in the reference
            raise IndexError("element/2 badarg on the empty ops tuple")
        first = tup.element(FIRST_OP + length)
        return (1, [(FIRST_OP, first)])
    return (new_size, new_ops)


def op_insert_gc(key, downstream_op: Payload, st: VnodeState):
    """:622-647."""
    if key not in st.ops_cache:
        st.ops_cache[key] = OpsTuple(key, 0, OPS_THRESHOLD, 0, [])
    t = st.ops_cache[key]
    t.elems[2] += 1
    new_id = t.elems[2]
    length, list_len = t.element(2)
    if length >= list_len or (new_id % OPS_THRESHOLD) == 0:
        internal_read(key, downstream_op.type, downstream_op.snapshot_time, IGNORE, True, st)
        t = st.ops_cache[key]
        new_length, new_list_len = t.element(2)
        _set_elem(t, new_length + FIRST_OP, (new_id, downstream_op))
        t.elems[1] = (new_length + 1, new_list_len)
    else:
        _set_elem(t, length + FIRST_OP, (new_id, downstream_op))
        t.elems[1] = (length + 1, list_len)
    return True


def _set_elem(t: OpsTuple, pos, v):
    if pos - 1 >= len(t.elems):
        raise IndexError("ets:update_element badarg")
    t.elems[pos - 1] = v


# ---------------------------------------------------------------------------
# GST: stable_time_functions + meta_data_sender
# ---------------------------------------------------------------------------
def update_func_min(last, time) -> bool:
    """src/stable_time_functions.erl:42-48."""
    if last == UNDEFINED:
        return True
    return time >= last


def get_min_time(d: dict) -> dict:
    """src/stable_time_functions.erl:51-85.  d: {Node/Partition: dict | UNDEFINED}."""
    min_dict: dict = {}
    found_undefined = False
    for _node, node_dict in d.items():
        if node_dict == UNDEFINED:
            found_undefined = True
            continue
        for dc, t in node_dict.items():
            prev = min_dict.get(dc, t)
            min_dict[dc] = t if prev >= t else prev
    if found_undefined:
        return {dc: 0 for dc in min_dict}
    return min_dict


def update_stable(last_result: dict, new_dict: dict, update_func=update_func_min):
    """src/meta_data_sender.erl:342-356."""
    changed = False
    acc = dict(last_result)
    for dc, t in new_dict.items():
        last = last_result.get(dc, UNDEFINED)
        if update_func(last, t):
            changed = True
            acc[dc] = t
    return changed, acc


def local_partition_dicts(partitions, local_table: dict, check_nodes: bool):
    """The partition bookkeeping of meta_data_sender:get_meta_data/3 (:269-339):
    with CheckNodes, partitions missing from the table read as 'undefined' and
    partitions no longer owned are dropped; without it the table is used as is."""
    if not check_nodes:
        return dict(local_table)
    return {p: local_table.get(p, UNDEFINED) for p in partitions}


def gst_gr(ss: dict) -> dict:
    """dc_utilities:get_stable_snapshot/0, txn_prot = gr (src/dc_utilities.erl:259-277)."""
    if not ss:
        return ss
    g = min(ss.values())
    return {k: g for k in ss}


# ---------------------------------------------------------------------------
# key -> partition (src/log_utilities.erl:60-118)
# ---------------------------------------------------------------------------
BUCKET = b"antidote"       # include/antidote.hrl:2


def chash_key(b: bytes) -> bytes:
    """riak_core_util:chash_key({?BUCKET, B}) = crypto:hash(sha, term_to_binary({<<"antidote">>, B}))
    for a binary B (SMALL_TUPLE_EXT of two BINARY_EXT; riak_core, un-vendored)."""
    import hashlib
    t2b = bytes([131, 104, 2, 109]) + len(BUCKET).to_bytes(4, "big") + BUCKET + bytes([109]) + \
        len(b).to_bytes(4, "big") + b
    return hashlib.sha1(t2b).digest()


def _list_to_integer(text: bytes):
    """erlang:list_to_integer/1 on a byte list: [+-]?[0-9]+, or None (badarg)."""
    i = 1 if text[:1] in (b"+", b"-") else 0
    if i == len(text) or not all(0x30 <= c <= 0x39 for c in text[i:]):
        return None
    v = int(text[i:].decode())
    return -v if text[:1] == b"-" else v


def convert_key(key, term_bytes: Optional[bytes] = None) -> int:
    """:100-118.  A key that is neither an integer nor a binary is given as term_to_binary(Key)
    (term_bytes)."""
    if isinstance(key, (bytes, Bin)):
        v = _list_to_integer(bytes(key))
        if v is not None:
            return abs(v)
        return abs(int.from_bytes(chash_key(bytes(key)), "big"))
    if isinstance(key, int):
        return abs(key)
    if term_bytes is None:
        raise ValueError("a non-integer, non-binary key needs its term_to_binary bytes")
    return abs(int.from_bytes(chash_key(term_bytes), "big"))


def get_partition_index(key, num_partitions: int) -> int:
    """1-based position into the sorted partition list (get_primaries_preflist/1, :76-79)."""
    return convert_key(key) % num_partitions + 1
