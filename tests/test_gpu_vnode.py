"""The device materializer_vnode (am_vnode: op_insert_gc/3 with its GC reads, internal_read/7
with the snapshot cache and snapshot_insert_gc/4) against

  * the reference's six vnode EUnit KATs (src/materializer_vnode.erl:652-852: gc_test,
    large_list_test, seq_write_test, multipledc_write_test, concurrent_write_test,
    read_nonexisting_key_test; transcribed in tests/golden/kat_vnode.json), and
  * the oracle's VnodeState (oracle/ref_materializer.py: op_insert_gc, internal_read,
    snapshot_insert_gc, prune_ops) on random multi-key sequences of every type.

Bar: every read value equal (LogColdPath <-> AM_ERR_COLD_PATH), and after every step the
whole state equal key by key: the ops-cache tuple header {Length, ListLen} and OpCounter, the
op ids in the cache, and the snapshot dict (clock, last_op_id, value, newest first)."""
import random

import pytest

from antidote_amd import abi
from antidote_amd.oplog import Op, Read
from oracle import ref_materializer as R
from tests import randlog
from tests.kat_util import load, payload

pytestmark = pytest.mark.gpu

VN = load("kat_vnode.json")


@pytest.fixture(scope="module")
def mat():
    from antidote_amd.materializer import Materializer
    m = Materializer(0)
    yield m
    m.close()


def _canon(t, v):
    return randlog.canon_state(t, v)


def compare_state(vn, st, keys, types, dcmap):
    """keys: device key -> oracle key; dcmap: oracle DC id -> device index."""
    for k, ok in keys.items():
        t = st.ops_cache.get(ok)
        length, list_len, counter = vn.key_info(k)
        if t is None:
            assert (length, list_len, counter) == (0, 0, 0), k
            assert vn.op_ids(k) == []
        else:
            rl, rll = t.element(2)
            assert (length, list_len, counter) == (rl, rll, t.element(3)), (k, (length, list_len, counter), (rl, rll))
            assert vn.op_ids(k) == [t.element(R.FIRST_OP + i)[0] for i in range(rl)], k
        sd = st.snapshot_cache.get(ok)
        dev = vn.snapshots(k, types[k])
        if sd is None:
            assert dev is None, k
            continue
        lst, size = sd
        assert dev is not None and len(dev) == size == len(lst), (k, dev, lst)
        for (clock, snap), (dclock, dlo, dval) in zip(lst, dev):
            assert {dcmap[d]: v for d, v in clock.items()} == dclock, (k, clock, dclock)
            assert snap.last_op_id == dlo, (k, snap.last_op_id, dlo)
            assert _canon(types[k], snap.value) == dval, (k, snap.value, dval)


def _kat_dcmap(actions):
    dcs = set()
    for a in actions:
        if a[0] == "insert":
            dcs.add(a[1]["commit"][0])
            dcs |= {d for d, _ in a[1]["ss"]}
        else:
            dcs |= {d for d, _ in a[1]}
    return {d: i for i, d in enumerate(sorted(dcs, key=lambda x: (isinstance(x, str), x)))}


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
def test_gpu_vnode_kat(mat, kat):
    """The EUnit test's actions through am_vnode_insert_host / am_vnode_read_host (consecutive
    inserts batched into one call), each read's value asserted as the reference asserts it,
    and the device state compared with the oracle's after every call."""
    actions = _large_list_actions() if kat.get("generator") == "large_list" else kat["actions"]
    m = _kat_dcmap(actions)
    t = kat["type"]
    vn = mat.vnode(max(len(m), 1), 1)
    st = R.VnodeState()
    try:
        i = 0
        while i < len(actions):
            a = actions[i]
            if a[0] == "insert":
                batch = []
                while i < len(actions) and actions[i][0] == "insert":
                    p = actions[i][1]
                    batch.append(Op(type=t, commit_dc=m[p["commit"][0]], commit_time=p["commit"][1],
                                    snap={m[d]: v for d, v in p["ss"]}, effect=p["param"], txid=p["txid"]))
                    R.op_insert_gc(kat["key"], payload(p, t, key=kat["key"]), st)
                    i += 1
                vn.insert([batch], [t])
            else:
                _, clock, gc, expect = a
                got = vn.read([Read(0, t, {m[d]: v for d, v in clock})], should_gc=[gc]).result(0)
                ref = R.internal_read(kat["key"], t, {d: v for d, v in clock}, R.IGNORE, gc, st)
                assert got[0] == "ok" and got[1] == expect == R.crdt_value(t, ref[1]), (i, a, got)
                i += 1
            compare_state(vn, st, {0: kat["key"]}, {0: t}, m)
    finally:
        vn.close()


class KeyGen:
    """A key's stream of causally plausible ops (randlog.rand_effect), clock moving forward."""

    def __init__(self, rng, t, n_dc, t0):
        self.rng, self.t, self.n_dc, self.clock, self.state = rng, t, n_dc, t0, {}

    def ops(self, n):
        # Snapshot entries trail the commit clock by a fixed LAG and the clock moves 2-4 per
        # op: snapshots are monotone, so a later op's snapshot covers every snapshot an earlier
        # GC read cached (op_insert_gc's GC reads never take the log cold path, which is not on
        # the device), and the last ~LAG/3 ops are never inside a GC read, so prune_ops keeps
        # them (when it keeps nothing the reference stores a placeholder its next read crashes
        # on -- src/materializer_vnode.erl:580-583 -- and such keys leave the comparison).
        out = []
        for _ in range(n):
            self.clock += self.rng.randint(2, 4)
            dc = self.rng.randrange(self.n_dc)
            snap = {d: max(0, self.clock - 20) for d in range(self.n_dc)}
            out.append(Op(type=self.t, commit_dc=dc, commit_time=self.clock, snap=snap,
                          effect=randlog.rand_effect(self.rng, self.t, self.n_dc, self.state)))
        return out


def _placeholder(st, k):
    """prune_ops kept element(FIRST_OP+Len) -- a 0 -- when it pruned every op
    (src/materializer_vnode.erl:580-583); the reference's next read of the key crashes on it
    (clocksi_materializer's {OpId, Op} match), so such keys leave the comparison."""
    t = st.ops_cache.get(k)
    return t is not None and t.element(2)[0] > 0 and t.element(R.FIRST_OP) == 0


def _oracle_payload(op, key):
    return randlog.payload_term(op, key=key)


@pytest.mark.parametrize("seed", range(3))
def test_gpu_vnode_random(mat, seed):
    """Random insert batches (1-70 ops per key: GC triggers every 50 ids and on full tuples)
    and read batches (repeated keys, ShouldGC on some reads, old clocks that take the log
    cold path) over keys of all five types, against the oracle's VnodeState."""
    rng = random.Random(9100 + seed)
    n_dc = [1, 3, 4][seed]
    types = [abi.AM_PN, abi.AM_LWW, abi.AM_AWSET, abi.AM_MVREG, abi.AM_BCOUNTER]
    n_keys = 20
    ktype = [types[k % 5] for k in range(n_keys)]
    gens = [KeyGen(rng, ktype[k], n_dc, 10 + rng.randint(0, 50)) for k in range(n_keys)]
    vn = mat.vnode(n_dc, n_keys)
    st = R.VnodeState()
    dcmap = {d: d for d in range(n_dc)}
    dead = set()  # keys whose reference tuple holds prune_ops' placeholder (a reference crash)
    try:
        for step in range(14):
            if step % 2 == 0:  # an insert batch
                batch = [[] for _ in range(n_keys)]
                for k in rng.sample(range(n_keys), 12):
                    if k in dead:
                        continue
                    batch[k] = gens[k].ops(rng.choice([1, 5, 30, 49, 70]))
                for k in range(n_keys):
                    for op in batch[k]:
                        if _placeholder(st, k):  # pruned empty by a GC read of this batch
                            dead.add(k)
                            break
                        R.op_insert_gc(k, _oracle_payload(op, k), st)
                vn.insert(batch, ktype)
            else:  # a read batch with repeated keys
                reads, sg = [], []
                for _ in range(30):
                    k = rng.randrange(n_keys)
                    if k in dead:
                        continue
                    c = gens[k].clock
                    q = rng.random()
                    at = c + 5 if q < 0.6 else (c - rng.randint(0, 40) if q < 0.9 else rng.randint(0, c))
                    reads.append(Read(k, ktype[k], {d: max(0, at + rng.randint(-2, 2)) for d in range(n_dc)}))
                    sg.append(rng.random() < 0.08)
                got = vn.read(reads, should_gc=sg, set_capacity=[4096] * len(reads))
                for i, rd in enumerate(reads):
                    if _placeholder(st, rd.key):  # a GC earlier in this batch pruned every op
                        dead.add(rd.key)
                    if rd.key in dead:
                        continue
                    try:
                        ref = R.internal_read(rd.key, rd.type, dict(rd.clock), R.IGNORE, sg[i], st)
                    except R.LogColdPath:
                        ref = ("cold",)
                    g = got.result(i)
                    if ref[0] == "cold":
                        assert g == ("error", abi.AM_ERR_COLD_PATH), (step, i, rd, g)
                    elif ref[0] == "error":
                        assert g[0] == "error", (step, i, rd, g, ref)
                    else:
                        assert g[0] == "ok" and g[1] == _canon(rd.type, ref[1]), (step, i, rd, g, ref)
            for k in range(n_keys):
                if _placeholder(st, k):
                    dead.add(k)
            compare_state(vn, st, {k: k for k in range(n_keys) if k not in dead}, ktype, dcmap)
    finally:
        vn.close()
