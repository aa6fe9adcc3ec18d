"""The oracle (oracle/ref_materializer.py) against the values the reference's multi-DC,
bounded-counter and staged-read system suites assert (tests/golden/multidc_suites.json), each
scenario replayed over one VnodeState per DC by tests/dcsim.py."""
import pytest

from tests import dcsim
from tests.kat_util import load

SUITES = load("multidc_suites.json")
SUITES["cases"] = SUITES["cases"] + load("txn_suites.json")["cases"]


@pytest.mark.parametrize("case", SUITES["cases"], ids=lambda c: c["name"])
def test_oracle_multidc_suite(case):
    checks = dcsim.run_case(case, lambda n_dc, keys: dcsim.OracleBackend(n_dc, keys))
    assert checks, "every case asserts something"
    for where, got, exp in checks:
        assert got == exp, where


def test_bcounter_permissions_restatement():
    # P: {dc0,dc0}:10 (increment), {dc0,dc1}:5 (transfer); D: {dc1}:5 -> 5 overall, 5 / 0 local
    st = ([((0, 0), 10), ((0, 1), 5)], [(1, 5)])
    assert dcsim.permissions(st) == 5
    assert dcsim.local_permissions(0, st) == 5 and dcsim.local_permissions(1, st) == 0
    # a transfer never changes the total
    assert dcsim.permissions(([((0, 0), 10), ((0, 1), 7)], [])) == 10
