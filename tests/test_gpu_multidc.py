"""The reference's multi-DC, bounded-counter and staged-read system-suite values
(tests/golden/multidc_suites.json) through the HIP path: one am_vnode per DC
(am_vnode_insert_host = op_insert_gc/3 for every local and replicated op, am_vnode_read_host =
materializer_vnode:read/6), the term codec for elements / values / tokens, the TxId map for
the reading transaction, and a transaction's own writes through am_materialize with TxId
inclusion (src/clocksi_materializer.erl:232).  Each scenario also runs on the oracle, and every
read the scenario makes must match it as a CRDT state, not only in the asserted value."""
import pytest

from tests import dcsim
from tests.kat_util import load

pytestmark = pytest.mark.gpu

SUITES = load("multidc_suites.json")
SUITES["cases"] = SUITES["cases"] + load("txn_suites.json")["cases"]


@pytest.fixture(scope="module")
def mat():
    from antidote_amd.materializer import Materializer
    m = Materializer(0)
    yield m
    m.close()


class _Tee:
    """Runs every backend call on the GPU and on the oracle and compares the states."""

    def __init__(self, n_dc, keys, mat):
        self.g = dcsim.GpuBackend(n_dc, keys, mat)
        self.o = dcsim.OracleBackend(n_dc, keys)
        self.n = 0

    def deliver(self, dc, ops):
        self.g.deliver(dc, ops)
        self.o.deliver(dc, ops)

    def read(self, dc, key, clock):
        a, b = self.g.read(dc, key, clock), self.o.read(dc, key, clock)
        assert a == b, ("read", dc, key, clock, a, b)
        self.n += 1
        return a

    def staged(self, dc, key, clock, txid, effects, base):
        a = self.g.staged(dc, key, clock, txid, effects, base)
        b = self.o.staged(dc, key, clock, txid, effects, base)
        assert a == b, ("staged", dc, key, clock, a, b)
        self.n += 1
        return a

    def restart(self, dc):
        self.g.restart(dc)
        self.o.restart(dc)

    def read_many(self, dc, keys, clock):
        a, b = self.g.read_many(dc, keys, clock), self.o.read_many(dc, keys, clock)
        assert a == b, ("read_many", dc, keys, clock, a, b)
        self.n += 1
        return a

    def gst(self, dc, parts, gr):
        a, b = self.g.gst(dc, parts, gr), self.o.gst(dc, parts, gr)
        assert a == b, ("gst", dc, parts, gr, a, b)
        return a

    def close(self):
        self.g.close()


@pytest.mark.parametrize("case", SUITES["cases"], ids=lambda c: c["name"])
def test_gpu_multidc_suite(mat, case):
    tees = []

    def factory(n_dc, keys):
        t = _Tee(n_dc, keys, mat)
        tees.append(t)
        return t

    checks = dcsim.run_case(case, factory)
    assert checks and tees[0].n > 0
    for where, got, exp in checks:
        assert got == exp, where


def test_gpu_txid_inclusion_with_pid_txids(mat):
    """An op the base snapshot already covers is a candidate only through TxId == Op.txid:
    with #tx_id{} terms holding pids (am_txid ids), the reading transaction's own op is
    applied and another transaction's is not."""
    from antidote_amd.etf import Atom, Pid
    from antidote_amd.oplog import Op
    from antidote_amd.txid import TxIds
    t = TxIds()
    mine = t.intern((Atom("tx_id"), 1_760_000_000_000_001, Pid("antidote@127.0.0.1", 87, 0, 3)))
    other = t.intern((Atom("tx_id"), 1_760_000_000_000_001, Pid("antidote@127.0.0.1", 88, 0, 3)))
    assert mine != other
    clock = {0: 500}
    ops = [(2, Op(type=dcsim.PN, commit_dc=0, commit_time=500, snap={0: 400}, effect=7, txid=mine)),
           (1, Op(type=dcsim.PN, commit_dc=0, commit_time=450, snap={0: 400}, effect=5, txid=other))]
    r = mat.materialize(dcsim.PN, mine, clock, ops, base_clock={0: 500}, base_value=100, n_dc=1)
    assert r[0] == "ok" and r[1] == 107 and r[5] == 1, r
    r = mat.materialize(dcsim.PN, None, clock, ops, base_clock={0: 500}, base_value=100, n_dc=1)
    assert r[0] == "ok" and r[1] == 100 and r[5] == 0, r
    t.close()
