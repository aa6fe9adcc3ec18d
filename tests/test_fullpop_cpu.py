"""CPU checks of the full-population parity harness (tests/fullpop.py): its vectorised oracle
batch gives the same results as the Read-by-Read HostBatch path, its comparator finds a single
changed output column or pair, and its chunking covers every key once."""
import numpy as np
import pytest

import bench
from antidote_amd import abi, synth
from antidote_amd.oplog import HostBatch, Read
from oracle import amo
from tests import fullpop, randlog


def _small(cfg_name, n_keys):
    cfg = dict(bench.CONFIGS[cfg_name])
    cfg["n_keys"] = n_keys
    if cfg.get("total_ops"):
        cfg["total_ops"] = n_keys * 64
        cfg["hot_cap"] = 2048
    return cfg, bench.synth_params(cfg)


def _as_dev(ref, kt, nk):
    dev = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in ref.items()}
    dev["_key_type"] = kt
    return dev


@pytest.mark.parametrize("cfg_name,esc", [("c2", 0), ("c3", 0), ("c4", 0), ("c5", 0), ("c4", 100000)])
def test_oracle_chunk_matches_hostbatch(cfg_name, esc):
    cfg, p = _small(cfg_name, 96 if cfg_name != "c3" else 24)
    p.esc_ppm = esc
    clock = synth.read_clock(p, bench.Q)
    cap = max(cfg["set_cap"], 1)
    k0, nk = 5, 17
    got = fullpop.oracle_chunk(p, k0, nk, clock, cap)
    hlog = synth.host_log(p, k0, nk)
    reads = [Read(k, int(hlog.key_type[k]), {d: clock[d] for d in range(p.n_dc)}) for k in range(nk)]
    ref = amo.materialize(hlog, HostBatch(p.n_dc, reads, randlog.caps_for(reads, p.n_dc, cap)))
    for i in range(nk):
        assert int(got["status"][i]) == int(ref.status[i])
        for c in fullpop.COMMON_COLS:
            assert int(got[c][i]) == int(getattr(ref, c)[i]), (c, i)
        assert (got["last_ct"][:, i] == ref.last_ct[:, i]).all()
        t = int(got["key_type"][i])
        if t in (abi.AM_AWSET, abi.AM_MVREG, abi.AM_BCOUNTER):
            o, n = int(got["set_off"][i]), int(got["set_len"][i])
            ro = int(ref.o_set_off[i])
            assert n == int(ref.o_set_len[i])
            assert (got["set_a"][o:o + n] == ref.o_set_a[ro:ro + n]).all()
            assert (got["set_b"][o:o + n] == ref.o_set_b[ro:ro + n]).all()
        for c in fullpop.VALUE_COLS.get(t, ()):
            assert int(got[c][i]) == int(getattr(ref, c)[i]), (c, i)


@pytest.mark.parametrize("cfg_name", ["c4", "c5"])
def test_compare_chunk_finds_single_changes(cfg_name):
    cfg, p = _small(cfg_name, 200)
    clock = synth.read_clock(p, bench.Q)
    cap = max(cfg["set_cap"], 1)
    nk = 200
    ref = fullpop.oracle_chunk(p, 0, nk, clock, cap)
    kt = ref["key_type"][:nk]
    dev = _as_dev(ref, kt, nk)
    assert len(fullpop.compare_chunk(dev, ref, 0, nk)) == 0
    sets = np.nonzero((ref["set_len"][:nk] > 0) & (ref["status"][:nk] == 0))[0]
    i = int(sets[len(sets) // 2])
    for col, mut in (("count", lambda d: d["count"].__setitem__(i, d["count"][i] + 1)),
                     ("last_ct", lambda d: d["last_ct"].__setitem__((0, i), d["last_ct"][0, i] ^ 1)),
                     ("pair", lambda d: d["set_b"].__setitem__(int(d["set_off"][i]) + int(d["set_len"][i]) - 1,
                                                                d["set_b"][int(d["set_off"][i]) + int(d["set_len"][i]) - 1] + 1)),
                     ("set_len", lambda d: d["set_len"].__setitem__(i, d["set_len"][i] - 1))):
        d = _as_dev(ref, kt, nk)
        mut(d)
        bad = fullpop.compare_chunk(d, ref, 0, nk)
        assert list(bad) == [i], (col, list(bad))


def test_chunks_cover_every_key_once():
    rng = np.random.default_rng(3)
    lens = rng.integers(0, 3000, 5000)
    lens[17] = 1 << 23  # a key above the chunk limit is a chunk alone
    parts = fullpop.chunks(len(lens), lens, max_ops=1 << 16, max_keys=64)
    seen = np.zeros(len(lens), int)
    for k0, nk in parts:
        assert nk >= 1 and (nk == 1 or lens[k0:k0 + nk].sum() <= 1 << 16) and nk <= 64
        seen[k0:k0 + nk] += 1
    assert (seen == 1).all()


def test_escape_knob_rate_and_shape():
    """bench.py --escape: about esc_ppm / 10^6 of the ops carry exactly one entry 2^33 us below
    the op's own timeline, never at the commit DC; esc_ppm = 0 leaves the log unchanged."""
    cfg, p = _small("c4", 4000)
    base = synth.host_log(p, 0, 4000)
    p.esc_ppm = 100000
    log = synth.host_log(p, 0, 4000)
    assert (log.commit_time == base.commit_time).all() and (log.p0 == base.p0).all()
    low = log.snap_vc < base.snap_vc  # [n_dc][n_ops]
    per_op = low.sum(axis=0)
    assert set(np.unique(per_op).tolist()) <= {0, 1}
    rate = per_op.mean()
    assert 0.08 < rate < 0.12, rate
    d = np.argmax(low, axis=0)[per_op == 1]
    cdc = (log.op_meta[:log.n_ops][per_op == 1] & 0x1F)
    assert (d != cdc).all()
    assert (base.snap_vc[low] - log.snap_vc[low] == 1 << 33).all()
