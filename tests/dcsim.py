"""A multi-DC AntidoteDB cluster for the reference's system-suite scenarios
(tests/golden/multidc_suites.json): one materializer vnode per DC holding one partition's keys,
transactions committed at a DC and replicated to the others in commit order, reads through
the vnode's read path.  Two backends run the same scenario:

  OracleBackend  oracle/ref_materializer.py's VnodeState (op_insert_gc/3, internal_read/7) and
                 materializer:materialize_eager/3 for a transaction's own writes
  GpuBackend     the HIP library: am_vnode_insert_host / am_vnode_read_host per DC, the term
                 codec for elements / values / tokens, the TxId map (am_txid) for the
                 reading transaction, and a transaction's own writes through am_materialize
                 with TxId inclusion (is_op_in_snapshot/7's `TxId == Op.txid`,
                 src/clocksi_materializer.erl:232)

Restated here (client side of the read path, not the path itself):
  * antidote_crdt downstream/2 (un-vendored, @4157110c): counter_pn increment/decrement -> N;
    set_aw add/remove -> [{E, [Token], Current}] / [{E, [], Current}] (the element's observed
    tokens, object_log_state_SUITE.erl:96-105 pins the fresh-element shape); register_mv
    assign -> {V, Token, CurrentTokens}; counter_b increment -> {{increment, N}, MyDC},
    decrement -> {{decrement, N}, MyDC} when localPermissions(MyDC) >= N else
    {error, no_permissions}, transfer {N, To, From} -> {{transfer, N, To}, From} (generated at
    src/bcounter_mgr.erl:80-97).
  * antidote_crdt_counter_b permissions/1 (the value the suites assert) = sum of the P entries
    {Id, Id} minus every D entry; localPermissions/2 = P entries into Id minus P entries out
    of Id minus D[Id].
  * bcounter_mgr's transfer protocol (src/bcounter_mgr.erl:111-205): a refused decrement
    queues Amount - Available; transfer_periodic asks the other DCs in ascending
    localPermissions order for the missing amount, and each transfers what it can.
  * clocksi_interactive_coord's reads inside a transaction: the snapshot read plus the
    transaction's own updates (apply_tx_updates_to_snapshot, src/clocksi_interactive_coord.erl:
    883-894).
Transactions at a DC snapshot at everything the DC has received (all DCs present in every
clock); a commit advances the DC's own entry.  Replication is immediate unless the scenario
holds it (concurrent writes) or disconnects a DC (failure_test); a held op is delivered before
any read or transaction whose clock needs it.
"""
from __future__ import annotations

import random
from typing import Any, Dict, List, Optional, Tuple

from oracle import ref_materializer as R

PN, LWW, AWSET, MVREG, BCOUNTER = R.PN, R.LWW, R.AWSET, R.MVREG, R.BCOUNTER
TYPES = {"counter_pn": PN, "register_lww": LWW, "set_aw": AWSET, "register_mv": MVREG, "counter_b": BCOUNTER}


class NoPermissions(Exception):
    pass


def jterm(x):
    """Fixture JSON -> Erlang term (atoms as str, binaries as bytes)."""
    if isinstance(x, dict):
        if "bin" in x:
            return x["bin"].encode()
        if "atom" in x:
            return str(x["atom"])
        if "seq" in x:
            a, b = x["seq"]
            return list(range(a, b + 1))
        raise ValueError(x)
    if isinstance(x, list):
        return [jterm(y) for y in x]
    return x


# ---- antidote_crdt_counter_b (un-vendored) restated over the P / D orddicts ----
def permissions(state) -> int:
    p, d = state
    return sum(v for (f, t), v in p if f == t) - sum(v for _, v in d)


def local_permissions(dc, state) -> int:
    p, d = state
    recv = sum(v for (f, t), v in p if t == dc)
    sent = sum(v for (f, t), v in p if f == dc and t != dc)
    dec = sum(v for i, v in d if i == dc)
    return recv - sent - dec


def crdt_value(type_, state):
    if type_ == BCOUNTER:
        return permissions(state)
    return R.crdt_value(type_, state)


# ---- antidote_crdt downstream/2 restated (effects over terms) ----
def downstream(type_, op, arg, state, dc, token):
    if type_ == PN:
        return int(arg) if op == "increment" else -int(arg)
    if type_ == LWW:
        raise NotImplementedError("no suite here assigns an LWW register")
    if type_ == AWSET:
        elems = [arg] if op in ("add", "remove") else list(arg)
        out = []
        for e in sorted(set(elems), key=_cmp_key):
            cur = next((toks for x, toks in state if R.erl_cmp(x, e) == 0), [])
            out.append((e, [token()] if op in ("add", "add_all") else [], list(cur)))
        return out
    if type_ == MVREG:
        return ("assign", arg, token(), [t for _, t in state])
    if type_ == BCOUNTER:
        if op == "increment":
            return ("increment", int(arg), dc)
        if op == "decrement":
            if local_permissions(dc, state) < int(arg):
                raise NoPermissions()
            return ("decrement", int(arg), dc)
        if op == "transfer":
            amount, to, frm = arg
            if local_permissions(frm, state) < amount:
                raise NoPermissions()
            return ("transfer", amount, to, frm)
    raise ValueError((type_, op))


class _Key:
    def __init__(self, t):
        self.t = t

    def __lt__(self, o):
        return R.erl_cmp(self.t, o.t) < 0


def _cmp_key(t):
    return _Key(t)


def _oracle_effect(type_, eff):
    if type_ == MVREG:
        return (eff[1], eff[2], list(eff[3])) if eff[0] == "assign" else ("reset", list(eff[1]))
    if type_ == BCOUNTER:
        if eff[0] == "transfer":
            return (("transfer", eff[1], eff[2]), eff[3])
        return ((eff[0], eff[1]), eff[2])
    return eff


def _bc_state(pd: Dict, dd: Dict):
    return (sorted(pd.items()), sorted(dd.items()))


class OracleBackend:
    name = "oracle"

    def __init__(self, n_dc, keys):
        self.n_dc, self.keys = n_dc, keys
        self.st = [R.VnodeState() for _ in range(n_dc)]
        self.log: List[List[Tuple]] = [[] for _ in range(n_dc)]   # the DC's logging_vnode, in commit order
        self.stable = [dict() for _ in range(n_dc)]               # meta_data_sender's last stable result

    def deliver(self, dc, ops):
        for key, type_, eff, snap, origin, ct, txid in ops:
            self.log[dc].append((key, type_, eff, snap, origin, ct, txid))
            p = R.Payload(key=key, type=type_, op_param=_oracle_effect(type_, eff), snapshot_time=dict(snap),
                          commit_time=(origin, ct), txid=txid)
            R.op_insert_gc(key, p, self.st[dc])

    def restart(self, dc):
        """Kill and restart the DC's node: the ops cache is gone and load_from_log_to_tables/2 ->
        load_ops/2 replays the log through op_insert_gc/3 (src/materializer_vnode.erl:288-319)."""
        log, self.log[dc] = self.log[dc], []
        self.st[dc] = R.VnodeState()
        self.deliver(dc, log)

    def read_many(self, dc, keys, clock):
        return [self.read(dc, k, clock) for k in keys]

    def gst(self, dc, parts, gr):
        """stable_time_functions:get_min_time/1 over the partitions' stable clocks, the monotone
        meta_data_sender:update_stable/3, and dc_utilities:get_stable_snapshot/0 (gr: the min
        broadcast to every DC)."""
        merged = R.get_min_time({i: dict(c) for i, c in enumerate(parts)})
        _, self.stable[dc] = R.update_stable(self.stable[dc], merged)
        return R.gst_gr(dict(self.stable[dc])) if gr else dict(self.stable[dc])

    def read(self, dc, key, clock):
        r = R.internal_read(key, self.keys[key], dict(clock), R.IGNORE, False, self.st[dc])
        assert r[0] == "ok", r
        return self._norm(self.keys[key], r[1])

    def staged(self, dc, key, clock, txid, effects, base):
        """apply_tx_updates_to_snapshot: materializer:materialize_eager/3 of the writes."""
        t = self.keys[key]
        s = R.materialize_eager(t, self._denorm(t, base), [_oracle_effect(t, e) for e in effects])
        return self._norm(t, s)

    @staticmethod
    def _norm(t, s):
        if t == BCOUNTER:
            return (sorted(s[0]), sorted(s[1]))
        return s

    @staticmethod
    def _denorm(t, s):
        return (list(s[0]), list(s[1])) if t == BCOUNTER else s

    def close(self):
        pass


class GpuBackend:
    name = "gpu"

    def __init__(self, n_dc, keys, mat):
        from antidote_amd.codec import Codec
        from antidote_amd.txid import TxIds
        self.n_dc, self.keys, self.mat = n_dc, keys, mat
        self.kidx = {k: i for i, k in enumerate(keys)}
        self.ktypes = [keys[k] for k in keys]
        self.vn = [mat.vnode(n_dc, len(keys)) for _ in range(n_dc)]
        self.codec = [Codec() for _ in range(n_dc)]
        self.txids = [TxIds() for _ in range(n_dc)]
        self.log: List[List[List[Any]]] = [[[] for _ in keys] for _ in range(n_dc)]  # per DC, per key, log order
        self.last = [None] * n_dc   # the device GST state per DC: (last_vc, last_pres)

    def _labels(self, dc, type_, eff):
        if type_ == BCOUNTER:
            return eff
        lab, rl = self.codec[dc].effect(type_, eff)
        if rl:  # the codec re-spread its labels: relabel what the vnode holds first (a NIF does this)
            old, new = self.codec[dc].take_relabel()
            self.vn[dc].relabel(old, new)
        return lab

    def deliver(self, dc, ops):
        from antidote_amd.oplog import Op
        per_key: List[List[Any]] = [[] for _ in self.keys]
        for key, type_, eff, snap, origin, ct, txid in ops:
            # an op's TxId is stamped with its commit time: the map drops it once stable (am_txid)
            per_key[self.kidx[key]].append(Op(type=type_, commit_dc=origin, commit_time=ct, snap=dict(snap),
                                              effect=self._labels(dc, type_, eff),
                                              txid=self.txids[dc].intern_op(txid, origin, ct) if txid is not None
                                              else None))
        for k, ops_k in enumerate(per_key):
            self.log[dc][k] += ops_k
        self.vn[dc].insert(per_key, self.ktypes)

    def restart(self, dc):
        """The vnode is destroyed and rebuilt from the log: Materializer.load_ops (am_vnode_insert_host
        of every logged op, load_ops/2)."""
        self.vn[dc].close()
        self.vn[dc] = self.mat.load_ops(self.n_dc, self.log[dc], self.ktypes)

    def read_many(self, dc, keys, clock):
        """One read batch over several keys at one snapshot (one am_vnode_read_host call, as
        read_objects batches a transaction's reads)."""
        from antidote_amd.oplog import Read
        hb = self.vn[dc].read([Read(self.kidx[k], self.keys[k], dict(clock)) for k in keys],
                              set_capacity=[4096] * len(keys))
        out = []
        for i, k in enumerate(keys):
            r = hb.result(i)
            assert r[0] == "ok", r
            out.append(self._terms(dc, self.keys[k], r[1]))
        return out

    def gst(self, dc, parts, gr):
        """The device GST path: am_gst_local_min over the partitions' stable clocks (one node: its
        lanes are the all-reduce's result) and am_gst_finalize (monotone update; gr broadcast)."""
        import numpy as np
        import torch

        from antidote_amd import abi
        nd, npart = self.n_dc, len(parts)
        vc = np.zeros((npart, nd), np.uint64)
        pres = np.zeros(npart, np.uint32)
        for i, c in enumerate(parts):
            for d, t in c.items():
                vc[i, d] = t
                pres[i] |= 1 << d
        if self.last[dc] is None:
            self.last[dc] = (torch.zeros(nd, dtype=torch.int64, device="cuda"),
                             torch.zeros(1, dtype=torch.int32, device="cuda"))
        d_vc = torch.from_numpy(vc.view(np.int64)).cuda()
        d_pres = torch.from_numpy(pres.view(np.int32)).cuda()
        lanes = torch.zeros(nd + 1, dtype=torch.int64, device="cuda")
        o_vc = torch.zeros(nd, dtype=torch.int64, device="cuda")
        o_p = torch.zeros(1, dtype=torch.int32, device="cuda")
        ch = torch.zeros(1, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        L, ctx = self.mat.L, self.mat.ctx
        abi.check(L.am_gst_local_min(ctx, nd, npart, d_vc.data_ptr(), d_pres.data_ptr(), None, lanes.data_ptr()),
                  "am_gst_local_min")
        abi.check(L.am_gst_finalize(ctx, nd, lanes.data_ptr(), self.last[dc][0].data_ptr(),
                                    self.last[dc][1].data_ptr(), 1 if gr else 0, o_vc.data_ptr(), o_p.data_ptr(),
                                    ch.data_ptr()), "am_gst_finalize")
        self.mat.sync()
        out, p = o_vc.cpu().numpy().view(np.uint64), int(o_p.item()) & 0xFFFFFFFF
        return {d: int(out[d]) for d in range(nd) if (p >> d) & 1}

    def _read_labels(self, dc, key, clock):
        from antidote_amd.oplog import Read
        hb = self.vn[dc].read([Read(self.kidx[key], self.keys[key], dict(clock))], set_capacity=[4096])
        r = hb.result(0)
        assert r[0] == "ok", r
        return r[1]

    def _terms(self, dc, t, v):
        if t == BCOUNTER:
            return _bc_state(*v)
        return self.codec[dc].value(t, v)

    def read(self, dc, key, clock):
        t = self.keys[key]
        return self._terms(dc, t, self._read_labels(dc, key, clock))

    def staged(self, dc, key, clock, txid, effects, base):
        """The transaction's own writes through materialize/4: base = the snapshot read at the
        transaction's clock, the writes as ops carrying the transaction's TxId and that clock
        (so le(X, base) holds and only TxId == Op.txid makes them candidates)."""
        from antidote_amd.oplog import Op
        t = self.keys[key]
        tid = self.txids[dc].intern(txid)
        labs = [self._labels(dc, t, e) for e in effects]  # may relabel: intern before reading the base
        base_lab = self._read_labels(dc, key, clock)
        ops = [(i + 1, Op(type=t, commit_dc=dc, commit_time=clock[dc], snap=dict(clock), effect=e, txid=tid))
               for i, e in enumerate(labs)]
        r = self.mat.materialize(t, tid, dict(clock), list(reversed(ops)), base_clock=dict(clock),
                                 base_value=self._base(t, base_lab), n_dc=self.n_dc)
        assert r[0] == "ok", r
        assert r[5] == len(effects), ("every own write is applied", r)
        return self._terms(dc, t, r[1])

    @staticmethod
    def _base(t, v):
        if t == LWW:
            return v
        return v

    def close(self):
        for v in self.vn:
            v.close()
        for c in self.codec:
            c.close()
        for x in self.txids:
            x.close()


class Txn:
    def __init__(self, cl: "Cluster", dc: int, clock: Optional[Dict[int, int]], now: bool = False):
        self.cl, self.dc = cl, dc
        cl.wait_for(dc, clock)
        self.snap = cl.view(dc, clock)
        if now:  # ClockSI: the snapshot time is the DC's physical clock, prepared commits below it
            self.snap[dc] = max(self.snap[dc], cl.now[dc])
        self.prepared: Optional[int] = None
        cl.txn_seq += 1
        # #tx_id{local_start_time, server_pid}: a pid of the DC's node
        from antidote_amd.etf import Atom, Pid
        self.txid = (Atom("tx_id"), 1_760_000_000_000_000 + cl.txn_seq, Pid(f"antidote@dc{dc}", 80 + cl.txn_seq, 0, 1))
        self.ws: Dict[str, List[Any]] = {}

    def read(self, key):
        base = self.cl.b.read(self.dc, key, self.snap)
        if self.ws.get(key):
            return self.cl.b.staged(self.dc, key, self.snap, self.txid, self.ws[key], base)
        return base

    def update(self, key, op, arg):
        t = self.cl.keys[key]
        eff = downstream(t, op, arg, self.read(key), self.dc, self.cl.token)
        self.ws.setdefault(key, []).append(eff)

    def prepare(self):
        """clocksi_iprepare: the commit time is fixed now, the writes become visible at commit."""
        self.cl.now[self.dc] += 10
        self.prepared = self.cl.now[self.dc]
        out = dict(self.snap)
        out[self.dc] = self.prepared
        return out

    def commit(self, abort=False):
        if abort or not self.ws:
            return dict(self.snap)
        return self.cl.commit(self.dc, self.snap, self.txid, self.ws, ct=self.prepared)


class Cluster:
    def __init__(self, backend, n_dc, keys, seed=0x5EED):
        self.b, self.n_dc, self.keys = backend, n_dc, keys
        self.rng = random.Random(seed)
        self.seen = [[0] * n_dc for _ in range(n_dc)]   # seen[d][o]: newest commit of origin o at d
        self.now = [1000 * (d + 1) for d in range(n_dc)]
        self.pending: List[List[Tuple]] = [[] for _ in range(n_dc)]   # per destination, commit order
        self.hold = False
        self.down = set()
        self.txn_seq = 0
        self.bc_queue: Dict[Tuple[int, str], List[int]] = {}
        self.partial: List[List[Tuple]] = [[] for _ in range(n_dc)]   # delivered, their txn not complete

    def token(self):
        return bytes(self.rng.getrandbits(8) for _ in range(20))

    def view(self, dc, clock=None):
        v = {o: self.seen[dc][o] for o in range(self.n_dc)}
        for o, t in (clock or {}).items():
            v[o] = max(v[o], t)
        return v

    def _deliver(self, dest, upto=None):
        """Deliver held ops to dest in commit order (all, or those with commit time <= upto[origin])."""
        keep, go = [], []
        for item in self.pending[dest]:
            origin, ct = item[4], item[5]
            if upto is None or ct <= upto.get(origin, 0):
                go.append(item)
            else:
                keep.append(item)
        self.pending[dest] = keep
        if go:
            self.b.deliver(dest, go)
        for item in go + self.partial[dest]:   # a partly delivered transaction is complete now
            self.seen[dest][item[4]] = max(self.seen[dest][item[4]], item[5])
        self.partial[dest] = []

    def deliver_some(self, dest, count):
        """Deliver the next `count` held ops to dest WITHOUT making their transaction visible
        (the DC's clock does not advance until the rest arrives): the ops sit in the ops cache,
        and a read at the DC's snapshot must exclude all of them (is_op_in_snapshot/7)."""
        go, self.pending[dest] = self.pending[dest][:count], self.pending[dest][count:]
        if go:
            self.b.deliver(dest, go)
            self.partial[dest] += go

    def wait_for(self, dc, clock):
        if clock:
            self._deliver(dc, clock)
            for o, t in clock.items():
                if self.seen[dc][o] < t:
                    raise AssertionError(f"DC {dc} cannot reach clock {clock}: disconnected")

    def flush(self):
        for d in range(self.n_dc):
            if d not in self.down:
                self._deliver(d)

    def commit(self, dc, snap, txid, ws, ct=None):
        if ct is None:
            self.now[dc] += 10
            ct = self.now[dc]
        items = [(key, self.keys[key], eff, dict(snap), dc, ct, txid) for key, effs in ws.items() for eff in effs]
        self.b.deliver(dc, items)
        self.seen[dc][dc] = ct
        for d in range(self.n_dc):
            if d != dc:
                self.pending[d] += items
        if not self.hold:
            self.flush()
        out = dict(snap)
        out[dc] = ct
        return out

    def read(self, dc, key, clock):
        self.wait_for(dc, clock)
        return self.b.read(dc, key, self.view(dc, clock))

    def gst_clock(self, dc, gr):
        """The DC's stable snapshot from its partitions' stable clocks (here the DC's one partition
        holds what it has applied)."""
        return self.b.gst(dc, [self.view(dc)], gr)

    # bcounter_mgr (src/bcounter_mgr.erl:111-205)
    def bc_refused(self, dc, key, amount):
        avail = local_permissions(dc, self.read(dc, key, None))
        if amount - avail:
            self.bc_queue.setdefault((dc, key), []).append(amount - avail)

    def bc_transfer_periodic(self, dc):
        for (d, key), q in list(self.bc_queue.items()):
            if d != dc or not q:
                continue
            required = sum(q)
            state = self.read(dc, key, None)
            prefs = sorted(((o, local_permissions(o, state)) for o in range(self.n_dc) if o != dc),
                           key=lambda x: x[1])
            remaining = required
            for remote, avail in prefs:
                if remaining > 0 and avail > 0:
                    req = remaining if avail - remaining >= 0 else avail
                    tx = Txn(self, remote, None)   # the remote DC's handle_cast({transfer, ...})
                    try:
                        tx.update(key, "transfer", (req, dc, remote))
                        tx.commit()
                    except NoPermissions:
                        pass
                    remaining -= req
            self.bc_queue[(d, key)] = [] if remaining == required else [remaining]


def _subst(x, env):
    if isinstance(x, str):
        for k, v in env.items():
            x = x.replace("{" + k + "}", str(v))
        if x.lstrip("-").isdigit() and any("{" + k + "}" in x for k in env):
            return int(x)
        return x
    if isinstance(x, list):
        return [_subst(y, env) for y in x]
    if isinstance(x, dict):
        return {k: _subst(v, env) for k, v in x.items()}
    return x


def _expand(steps, env=None):
    env = env or {}
    for s in steps:
        if "foreach" in s:
            f = s["foreach"]
            a, b = f["range"]
            for v in range(a, b + 1):   # {N} and {N-1}
                yield from _expand(f["steps"], dict(env, **{f["var"]: v, f["var"] + "-1": v - 1}))
        else:
            yield _subst_step(s, env)


def _subst_step(s, env):
    out = {}
    for k, v in s.items():
        if isinstance(v, dict):
            v = {kk: (_num(_subst(vv, env)) if kk in ("dc",) else _subst_arg(vv, env)) for kk, vv in v.items()}
        out[k] = v
    return out


def _num(x):
    return int(x) if isinstance(x, str) else x


def _subst_arg(v, env):
    if isinstance(v, str) and v.startswith("{") and v.endswith("}") and v[1:-1] in env:
        return env[v[1:-1]]
    if isinstance(v, list):
        return [_subst_arg(y, env) for y in v]
    if isinstance(v, str):
        for k, val in env.items():
            v = v.replace("{" + k + "}", str(val))
    return v


def run_case(case, backend_factory) -> List[Tuple[str, Any, Any]]:
    """Run one fixture case; returns the (where, got, expected) of every asserted read."""
    keys = {k: TYPES[t] for k, t in case["keys"].items()}
    b = backend_factory(case["n_dc"], keys)
    cl = Cluster(b, case["n_dc"], keys)
    clocks: Dict[str, Dict[int, int]] = {}
    txns: Dict[str, Txn] = {}
    checks = []
    clk = lambda name: None if name is None else clocks[name]  # noqa: E731
    try:
        for i, s in enumerate(_expand(case["steps"])):
            where = f"{case['name']} step {i}: {s}"
            if "txn" in s:
                a = s["txn"]
                tx = Txn(cl, a["dc"], clk(a.get("clock")))
                try:
                    for key, op, arg in a["updates"]:
                        tx.update(key, op, jterm(arg))
                except NoPermissions:
                    assert a.get("expect_error") == "no_permissions", where
                    for key, op, arg in a["updates"]:
                        if op == "decrement":
                            cl.bc_refused(a["dc"], key, int(arg))
                    checks.append((where, "no_permissions", "no_permissions"))
                    continue
                assert "expect_error" not in a, where + ": the update was not refused"
                ct = tx.commit()
                if "save" in a:
                    clocks[a["save"]] = ct
            elif "begin" in s:
                a = s["begin"]
                txns[a["name"]] = Txn(cl, a["dc"], clk(a.get("clock")), now=a.get("at") == "now")
            elif "prepare" in s:
                a = s["prepare"]
                ct = txns[a["txn"]].prepare()
                if "save" in a:
                    clocks[a["save"]] = ct
            elif "t_read" in s:
                a = s["t_read"]
                tx = txns[a["txn"]]
                st = tx.read(a["key"])
                checks.append((where, crdt_value(keys[a["key"]], st), jterm(a["expect"])))
            elif "t_update" in s:
                a = s["t_update"]
                txns[a["txn"]].update(a["key"], a["op"], jterm(a["arg"]))
            elif "commit" in s:
                a = s["commit"]
                ct = txns.pop(a["txn"]).commit(abort=a.get("abort", False))
                if "save" in a:
                    clocks[a["save"]] = ct
            elif "read" in s:
                a = s["read"]
                if a.get("at") in ("gst", "gst_gr"):   # a read at the stable snapshot itself
                    snap = cl.gst_clock(a["dc"], a["at"] == "gst_gr")
                    st = b.read(a["dc"], a["key"], snap)
                else:
                    snap = cl.view(a["dc"], clk(a.get("clock")))
                    st = cl.read(a["dc"], a["key"], clk(a.get("clock")))
                if "expect" in a:
                    checks.append((where, crdt_value(keys[a["key"]], st), jterm(a["expect"])))
                if "save" in a:
                    clocks[a["save"]] = dict(snap)
            elif "read_objects" in s:   # one batch, one snapshot
                a = s["read_objects"]
                cl.wait_for(a["dc"], clk(a.get("clock")))
                vals = [crdt_value(keys[k], x) for k, x in
                        zip(a["keys"], b.read_many(a["dc"], a["keys"], cl.view(a["dc"], clk(a.get("clock")))))]
                if "expect" in a:
                    checks.append((where, vals, jterm(a["expect"])))
            elif "deliver" in s:
                a = s["deliver"]
                cl.deliver_some(a["dc"], a["count"])
            elif "restart" in s:
                b.restart(s["restart"]["dc"])
            elif "hold" in s:
                cl.hold = s["hold"]
                if not cl.hold:
                    cl.flush()
            elif "disconnect" in s:
                cl.down.add(s["disconnect"]["dc"])
            elif "reconnect" in s:
                cl.down.discard(s["reconnect"]["dc"])
                cl.flush()
            elif "merge" in s:
                a = s["merge"]
                m: Dict[int, int] = {}
                for name in a["clocks"]:
                    for o, t in clocks[name].items():
                        m[o] = max(m.get(o, 0), t)
                clocks[a["save"]] = m
            elif "bc_transfer_periodic" in s:
                cl.bc_transfer_periodic(s["bc_transfer_periodic"]["dc"])
            else:
                raise ValueError(s)
    finally:
        b.close()
    return checks
