"""The reference's system-suite values for the read path, through the HIP path with real
Erlang terms: binaries, 20-byte binary tokens and integers go through the term codec
(am_codec) into the device's u64 labels, every transaction's effect through
am_vnode_insert_host (op_insert_gc/3), every read through am_vnode_read_host
(materializer_vnode:read/6 -> internal_read/7 -> materialize/4), and the labels back to
terms.  Fixtures: tests/golden/system_suites.json (pb_client_SUITE.erl:186-202, 237-321;
object_log_state_SUITE.erl:65-106).

The clients' downstream step (antidote_crdt:downstream/2, not on the read path) is restated
here: add -> [{E, [Token], []}], add_all -> an entry per element, LWW assign -> {Ts, V}, MV
assign -> {V, Token, Tokens of the current state}, increment -> N; tokens are fresh
20-byte binaries, as the suites' is_binary(Binary) assertions expect."""
import json
import os

import pytest

from antidote_amd import abi
from antidote_amd.codec import Codec
from antidote_amd.oplog import Op, Read

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
SUITES = json.load(open(os.path.join(HERE, "golden", "system_suites.json")))
TYPES = {"set_aw": abi.AM_AWSET, "register_lww": abi.AM_LWW, "register_mv": abi.AM_MVREG, "counter_pn": abi.AM_PN}


def _term(x):
    if isinstance(x, dict):
        return x["bin"].encode()
    if isinstance(x, list):
        return [_term(y) for y in x]
    return x


@pytest.fixture(scope="module")
def mat():
    from antidote_amd.materializer import Materializer
    m = Materializer(0)
    yield m
    m.close()


class Client:
    """One key on a one-DC partition: transactions commit in order, each read at the latest
    commit (start_transaction(ignore) after the previous commit)."""

    def __init__(self, mat, type_):
        self.t, self.codec, self.vn = type_, Codec(), mat.vnode(1, 1)
        self.clock, self.n = 1000, 0

    def close(self):
        self.vn.close()
        self.codec.close()

    def state(self):
        """The materialized state over terms at the latest commit."""
        hb = self.vn.read([Read(0, self.t, {0: self.clock})], set_capacity=[4096])
        r = hb.result(0)
        assert r[0] == "ok", r
        return self.codec.value(self.t, r[1])

    def downstream(self, upd):
        op, arg = upd[0], _term(upd[1])
        if self.t == abi.AM_AWSET:
            elems = [arg] if op == "add" else list(arg)
            return [(e, [os.urandom(20)], []) for e in elems]
        if self.t == abi.AM_LWW:
            return (self.clock * 1000 + 1, arg)
        if self.t == abi.AM_MVREG:
            cur = self.state() if self.n else []
            return ("assign", arg, os.urandom(20), [tok for _, tok in cur])
        return int(arg)

    def commit(self, updates):
        snap = self.clock
        self.clock += 10
        ops = []
        for u in updates:
            eff, rl = self.codec.effect(self.t, self.downstream(u))
            if rl:  # the codec ran out of gap labels: relabel what the vnode holds, as a NIF would
                old, nw = self.codec.take_relabel()
                self.vn.relabel(old, nw)
            ops.append(Op(type=self.t, commit_dc=0, commit_time=self.clock, snap={0: snap}, effect=eff))
        self.vn.insert([ops], [self.t])
        self.n += len(ops)
        return self.clock


def _value(t, state):
    if t == abi.AM_AWSET:
        return [e for e, _ in state]
    if t == abi.AM_LWW:
        return state[1]
    if t == abi.AM_MVREG:
        return [v for v, _ in state]
    return state


@pytest.mark.parametrize("case", [c for c in SUITES["cases"] if "txns" in c], ids=lambda c: c["name"])
def test_gpu_pb_client_suite_values(mat, case):
    t = TYPES[case["type"]]
    cl = Client(mat, t)
    try:
        for txn in case["txns"]:
            cl.commit(txn)
        v = _value(t, cl.state())
        exp = case["expect"]
        if "value" in exp:
            assert v == _term(exp["value"]), (case["name"], v)
        if "length" in exp:
            assert len(v) == exp["length"] and all(_term(x) in v for x in exp["contains"]), v
    finally:
        cl.close()


def test_gpu_object_log_state_suite(mat):
    case = next(c for c in SUITES["cases"] if c["name"] == "object_log_state_test")
    cl = Client(mat, abi.AM_AWSET)
    try:
        commit1 = None
        for ph in case["phases"]:
            lo, hi = ph["add_each"]
            for i in range(lo, hi + 1):  # add_set/4: one transaction per element
                c = cl.commit([["add", i]])
            st = cl.state()
            exp = ph["expect"]
            a, b = exp["value_seq"]
            assert [e for e, _ in st] == list(range(a, b + 1))
            if exp.get("state_one_binary_token_each"):  # check_orset_state/2
                assert all(len(toks) == 1 and isinstance(toks[0], bytes) and len(toks[0]) == 20 for _, toks in st)
            if "log_ops_after_first_phase" in exp:  # check_orset_ops/3 over the ops cache
                a, b = exp["log_ops_after_first_phase"]
                d = cl.vn.store().download()
                ko, vo, vd = d["key_off"], d["var_off"], d["var_data"]
                got = []
                for p in range(int(ko[0]), int(ko[1])):
                    if int(d["commit_time"][p]) <= commit1:
                        continue
                    w = [int(x) for x in vd[int(vo[p]):int(vo[p + 1])]]
                    assert w[1:3] == [1, 0], w  # one entry: one add token, no removes
                    got.append((cl.codec.term(w[0]), cl.codec.term(w[3]), []))
                assert [g[0] for g in got] == list(range(a, b + 1))
                assert all(isinstance(g[1], bytes) and len(g[1]) == 20 for g in got)
            commit1 = c
    finally:
        cl.close()
