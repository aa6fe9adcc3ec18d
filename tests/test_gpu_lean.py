"""The batch-clock ("lean") kernels' escape paths at D = 16: ops outside the packed view (here
ops with an invalid effect, AM_META_BAD, which the packed view escapes) evaluated from the full
columns one DC at a time, with their LastOpCt maxima through LDS -- k_bc_wave<16, false>
(bounded counter, 65..4096 ops), k_big_run / k_big_gincl (bounded counter above 4096 ops, MV
keys in the chunked big view).  One batch clock for every read (DeviceReads: per_read_clock 0,
the path these kernels take), checked against the oracle on every key."""
import random

import numpy as np
import pytest
import torch

from antidote_amd import abi
from antidote_amd.devbatch import DeviceReads, materialize
from antidote_amd.oplog import HostBatch, HostLog, Read
from oracle import amo
from tests import randlog

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mat():
    from antidote_amd.materializer import Materializer
    m = Materializer(0)
    yield m
    m.close()


@pytest.mark.parametrize("t,lens", [(abi.AM_BCOUNTER, [3, 40, 70, 300, 900, 2500, 5000, 6000]),
                                    (abi.AM_MVREG, [3, 30, 200, 1100, 1500, 3000])])
@pytest.mark.parametrize("bad_rate", [0.0, 0.004])
def test_gpu_batch_clock_escaped_ops_d16(mat, t, lens, bad_rate):
    rng = random.Random(4242 + t + int(bad_rate * 1000))
    n_dc = 16
    keys = []
    for i in range(2 * len(lens)):
        keys.append(randlog.rand_key_ops(rng, t, n_dc, lens[i % len(lens)], bad_rate=bad_rate,
                                         t0=rng.randint(0, 100)))
    log = HostLog(n_dc, keys, key_types=[t] * len(keys))
    st = mat.store(log)
    dlog = st.device_log()
    hi = max(op.commit_time for ops in keys for op in ops)
    clock = [int(hi * 0.75)] * n_dc
    n = len(keys)
    dr = DeviceReads(n, n_dc, t, clock, set_cap=512)
    torch.cuda.synchronize()
    materialize(mat, dlog, dr)
    mat.sync()
    h = dr.host()
    reads = [Read(k, t, {d: clock[d] for d in range(n_dc)}) for k in range(n)]
    ref = amo.materialize(log, HostBatch(n_dc, reads, randlog.caps_for(reads, n_dc, 512)))
    ok = [i for i in range(n) if ref.result(i)[0] == "ok"]
    vals = dr.values(np.asarray(ok, np.int64)) if ok else []
    for i in range(n):
        r = ref.result(i)
        if r[0] != "ok":
            assert int(h["status"][i]) == r[1], (i, int(h["status"][i]), r)
            continue
        assert int(h["status"][i]) == 0, (i, int(h["status"][i]), r)
        ct = None if h["last_ct_ignore"][i] else {d: int(h["last_ct"][d, i]) for d in range(n_dc)
                                                  if (int(h["last_ct_pres"][i]) >> d) & 1}
        got = ("ok", vals[ok.index(i)], int(h["new_last_op"][i]), ct, bool(h["is_new_ss"][i]), int(h["count"][i]),
               int(h["flags"][i]))
        assert got == r, (i, len(keys[i]), got, r)
    if bad_rate:
        assert any(ref.result(i)[0] != "ok" for i in range(n)), "no included invalid effect: the escape path is idle"
    st.close()
