"""BASELINE.json configs at their FULL bench sizes (bench.CONFIGS: C2 1M keys x 256 ops, C3
1M x 1024, C4 8M x 16, C5 2M keys / 1.34e8 Zipf ops after the 2^20 hot-key cap), read exactly as bench.py reads them
(one batch over every key of the GPU at the q = 0.75 clock).  Size-independent properties on
every read (status ok, Count <= the key's ops, LastOpCt within the read clock), and
bit-exact parity with the oracle on keys sampled across the whole key space -- eight
ranges of 32 keys spread over the store plus the longest logs -- regenerated on the host
(the counter-based generator is bit-identical per key)."""
import numpy as np
import pytest
import torch

import bench
from antidote_amd import abi, synth
from antidote_amd.devbatch import DeviceReads, materialize
from antidote_amd.oplog import HostBatch, Read
from oracle import amo
from tests import randlog

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mat():
    from antidote_amd.materializer import Materializer
    m = Materializer(0)
    yield m
    m.close()


def _ranges(n_keys, hot):
    """eight ranges of 32 keys spread over the key space, and each of the longest logs alone"""
    per = 32
    spread = [(int(x), per) for x in np.linspace(0, n_keys - per, 8)]
    return spread + [(int(h), 1) for h in hot if not any(s <= int(h) < s + n for s, n in spread)]


@pytest.mark.parametrize("cfg_name,index", [("c2", 3), ("c3", 3), ("c3", 0), ("c4", 3), ("c5", 3)],
                         ids=["c2", "c3", "c3-stream", "c4", "c5"])
def test_fullsize_config(mat, cfg_name, index):
    """index: the store's zone index (am_store_index level; 0 = none, every op streamed: the bench
    headline's store)."""
    cfg = bench.CONFIGS[cfg_name]
    p = bench.synth_params(cfg)
    st = mat.synth_store(p)
    try:
        if index != 3:
            st.index(index)
        dlog = st.device_log()
        ko, kt = bench.key_columns(mat, dlog, p.n_keys)
        clock = synth.read_clock(p, bench.Q)
        type_ = cfg["type"]
        mixed = type_ not in range(1, 6)
        cap = max(cfg["set_cap"], 1)
        dr = DeviceReads(p.n_keys, p.n_dc, 0 if mixed else type_, clock, set_cap=cap,
                         types=torch.from_numpy(kt.copy()).cuda() if mixed else None)
        torch.cuda.synchronize()
        materialize(mat, dlog, dr)
        mat.sync()
        h = dr.host()
        # ---- properties of every read ----
        assert (h["status"] == 0).all(), np.unique(h["status"], return_counts=True)
        lens = np.diff(ko.astype(np.int64))
        assert (h["count"].astype(np.int64) <= lens).all()
        pres = h["last_ct_pres"].astype(np.int64)
        for d in range(p.n_dc):
            has = ((pres >> d) & 1).astype(bool) & (h["last_ct_ignore"] == 0)
            assert (h["last_ct"][d][has] <= np.uint64(clock[d])).all(), d
        assert ((h["count"] > 0) == (h["is_new_ss"] != 0)).all()
        # ---- bit-exact parity on sampled key ranges ----
        hot = np.argsort(-lens)[:4]
        for k0, nk in _ranges(p.n_keys, hot):
            while nk > 1 and lens[k0:k0 + nk].sum() > (1 << 21):  # bound the host regeneration
                nk -= 1
            hlog = synth.host_log(p, k0, nk)
            reads = [Read(k, int(hlog.key_type[k]), {d: clock[d] for d in range(p.n_dc)}) for k in range(nk)]
            ref = amo.materialize(hlog, HostBatch(p.n_dc, reads, randlog.caps_for(reads, p.n_dc, cap)))
            idx = np.arange(k0, k0 + nk)
            vals = dr.values(idx)
            for j, i in enumerate(idx):
                ct = None if h["last_ct_ignore"][i] else {d: int(h["last_ct"][d, i]) for d in range(p.n_dc)
                                                          if (int(h["last_ct_pres"][i]) >> d) & 1}
                got = ("ok", vals[j], int(h["new_last_op"][i]), ct, bool(h["is_new_ss"][i]), int(h["count"][i]),
                       int(h["flags"][i]))
                assert got == ref.result(j), (cfg_name, int(i), got, ref.result(j))
        del dr
    finally:
        st.close()
        torch.cuda.empty_cache()
