"""Pin the Python restatement (oracle/ref_materializer.py) to every known-answer test the
reference's EUnit suites hold for the hot path (transcribed under tests/golden/)."""
import pytest

from oracle import ref_materializer as R
from tests.kat_util import load, payload, term, vc

KAT = load("kat_materialize.json")
VN = load("kat_vnode.json")


def _resp(ops, base):
    return R.SnapshotGetResponse(ops_list=ops, number_of_ops=len(ops),
                                 materialized_snapshot=R.MatSnapshot(base["last_op"], base["value"]),
                                 snapshot_time=base["ct"], is_newest_snapshot=True)


@pytest.mark.parametrize("kat", KAT["materialize"], ids=lambda k: k["name"])
def test_materialize_kat(kat):
    ops = [(i, payload(p, kat["type"])) for i, p in kat["ops"]]
    outs = []
    for case in kat["cases"]:
        if "base_from" in case:
            prev = outs[case["base_from"]]
            base = {"ct": prev[3], "last_op": prev[2], "value": prev[1]}
        else:
            b = case["base"]
            base = {"ct": vc(b["ct"]), "last_op": b["last_op"], "value": b["value"]}
        r = R.materialize(kat["type"], R.IGNORE if case["txid"] is None else case["txid"],
                          vc(case["read"]), _resp(ops, base))
        assert r[0] == "ok"
        outs.append(r)
        exp = case["expect"]
        assert r[1] == exp["value"]
        if "new_last_op" in exp:
            assert r[2] == exp["new_last_op"]
        if "last_op_ct" in exp:
            assert r[3] == vc(exp["last_op_ct"])
        if "is_new_ss" in exp:
            assert r[4] == exp["is_new_ss"]
        if "count" in exp:
            assert r[5] == exp["count"]
        if "intern_first_hole" in case:   # materialize_intern called directly in the reference test
            ri = R.materialize_intern(kat["type"], [], 0, case["intern_first_hole"], R.IGNORE,
                                      vc(case["read"]), ops, R.IGNORE, R.IGNORE, False, 0)
            assert ri == ("ok", [], exp["new_last_op"], R.IGNORE, False)


def test_materialize_intern_concurrent_kat():
    """materialize_intern called directly (src/clocksi_materializer.erl:413-418)."""
    kat = [k for k in KAT["materialize"] if k["name"] == "materializer_clocksi_concurrent_test"][0]
    ops = [(i, payload(p, kat["type"])) for i, p in kat["ops"]]
    ok, op_list, hole, ct, keep = R.materialize_intern(1, [], 0, 3, R.IGNORE, vc([[2, 2], [1, 2]]),
                                                       ops, R.IGNORE, R.IGNORE, False, 0)
    assert hole == 3 and ct == {1: 2, 2: 2}
    assert R.apply_operations(1, 0, 0, op_list)[1] == 4


def test_is_op_in_snapshot_kat():
    k = KAT["is_op_in_snapshot"][0]
    op = R.Payload("abc", 1, ("increment", 2), vc(k["op"]["ss"]), tuple(k["op"]["commit"]), k["op"]["txid"])
    for case in k["cases"]:
        r = R.is_op_in_snapshot(case["txid"], op, op.commit_time, op.snapshot_time, vc(case["read"]),
                                R.IGNORE, R.IGNORE)
        exp = case["expect"]
        assert r == (exp[0], exp[1], vc(exp[2]))


@pytest.mark.parametrize("case", KAT["belongs_to_snapshot_op"])
def test_belongs_to_snapshot_op_kat(case):
    assert R.belongs_to_snapshot_op(vc(case["ss"]), tuple(case["commit"]), vc(case["op_ss"])) == case["expect"]


@pytest.mark.parametrize("case", KAT["materialize_eager"])
def test_materialize_eager_kat(case):
    effects = [term(e) for e in case["effects"]]
    r = R.materialize_eager(case["type"], R.crdt_new(case["type"]), effects)
    if "expect_error" in case:
        assert r == ("error", term(case["expect_error"]))
    else:
        assert r == case["expect"]


def _run_vnode(kat, actions):
    st = R.VnodeState()
    for a in actions:
        if a[0] == "insert":
            R.op_insert_gc(kat["key"], payload(a[1], kat["type"], key=kat["key"]), st)
        else:
            _, clock, gc, expect = a
            r = R.internal_read(kat["key"], kat["type"], vc(clock), R.IGNORE, gc, st)
            assert r[0] == "ok"
            assert R.crdt_value(kat["type"], r[1]) == expect, a
    return st


def _large_list_actions():
    acts = [["read", [[1, 2]], False, 0]]
    for val in range(1, 1001):
        acts.append(["insert", {"ss": [[1, 10]], "commit": [1, 11 + val], "param": 1, "txid": 1}])
    acts.append(["read", [[1, 2000]], False, 1000])
    for val in range(1001, 1101):
        acts.append(["insert", {"ss": [[1, 10 + val]], "commit": [1, 11 + val], "param": 1, "txid": 1}])
        acts.append(["read", [[1, 2000]], False, val])
    return acts


@pytest.mark.parametrize("kat", VN["vnode"], ids=lambda k: k["name"])
def test_vnode_kat(kat):
    actions = _large_list_actions() if kat.get("generator") == "large_list" else kat["actions"]
    _run_vnode(kat, actions)


def test_vector_orddict_kat():
    v = VN["vector_orddict"]
    d0 = R.vo_new()
    d = d0
    for clock, val in v["dict3_inserts"]:
        d = R.vo_insert(vc(clock), val, d)
    dicts = {"empty": d0, "dict3": d}
    for name, ident, t, exp in v["get_smaller_from_id"]:
        r = R.vo_get_smaller_from_id(ident, t, dicts[name])
        assert (r == R.UNDEFINED) if exp is None else (r[1] == exp)
    for clock, exp_val, exp_first in v["get_smaller"]:
        r, first = R.vo_get_smaller(vc(clock), d)
        assert first == exp_first
        assert (r == R.UNDEFINED) if exp_val is None else (r[1] == exp_val)
    vb = R.vo_new()
    for clock, val, size in v["insert_bigger"]:
        vb = R.vo_insert_bigger(vc(clock), val, vb)
        assert vb[1] == size
    fl = R.vo_filter(lambda e: R.vc_gt(e[0], {}), ([(vc(c), s) for c, s in v["filter_list"]], 3))
    assert [s for _, s in fl[0]] == v["filter_gt_new_expect"]
    fdict = ([(vc(c), s) for c, s in v["filter_list"]], 3)
    for clock, exp in v["conc"]:
        assert R.vo_is_concurrent_with_any(fdict, vc(clock)) == exp


@pytest.mark.parametrize("case", VN["gst"], ids=lambda c: c["name"])
def test_gst_kat(case):
    table = {p: vc(c) for p, c in case["table"].items()}
    local = R.local_partition_dicts(case["partitions"], table, case["check_nodes"])
    assert R.get_min_time(local) == vc(case["expect"])


def test_convert_key_kat():
    for k, exp in VN["convert_key"]["cases"]:
        if isinstance(k, str) and k.startswith("b:"):
            k = R.Bin(k[2:].encode())
        assert R.convert_key(k) == exp


def test_update_stable_monotone():
    """update_stable keeps the larger of last/new per DC (src/meta_data_sender.erl:342-356)."""
    changed, res = R.update_stable({"a": 5, "b": 7}, {"a": 6, "b": 3, "c": 1})
    assert changed and res == {"a": 6, "b": 7, "c": 1}
    changed, res = R.update_stable({"a": 5}, {"a": 4})
    assert not changed and res == {"a": 5}
