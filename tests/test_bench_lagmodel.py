"""bench.py's layout-byte model: which reads are counted at the lag view's size (bench.lag_keys /
lag_split, DESIGN.md section 2 "Lag view"), on synthetic key columns -- no device needed."""
from types import SimpleNamespace

import numpy as np

import bench
from antidote_amd import abi


def _log(lag=True, gmask=True):
    return SimpleNamespace(lag_ct=1 if lag else 0, gmask=1 if gmask else 0, key_ngrp=0, rec_key_off=0, n_var=0)


def test_lag_split_configs():
    dl = _log()
    assert bench.lag_split(bench.CONFIGS["c3"], dl, abi.AM_INDEX_NONE)
    assert bench.lag_split(bench.CONFIGS["c4"], dl, abi.AM_INDEX_NONE)
    assert bench.lag_split(bench.CONFIGS["c5"], dl, abi.AM_INDEX_NONE)
    assert not bench.lag_split(bench.CONFIGS["c2"], dl, abi.AM_INDEX_NONE)  # LWW stream / row tiers
    assert not bench.lag_split(bench.CONFIGS["c3"], dl, abi.AM_INDEX_SUMMARIES)  # zone-indexed reads
    assert not bench.lag_split(bench.CONFIGS["c3"], _log(lag=False), abi.AM_INDEX_NONE)
    assert not bench.lag_split(dict(bench.CONFIGS["c3"], n_dc=32), dl, abi.AM_INDEX_NONE)


def test_lag_keys_single_type_set_config_is_every_key():
    kt = np.full(10, abi.AM_AWSET, np.uint8)
    ko = np.arange(0, 11 * 1024, 1024, dtype=np.uint64)
    assert bench.lag_keys(bench.CONFIGS["c3"], _log(), ko, kt, None).all()


def test_lag_keys_mixed_tiers():
    # key: type, ops, aligned start -> whether its tier streams the lag view
    cases = [(abi.AM_PN, 16, True),          # lane quad
             (abi.AM_LWW, 20, False),        # longer than a quad: the lane's own packed scan
             (abi.AM_MVREG, 12, True),       # quad (groups <= 32 with the group-mask view)
             (abi.AM_MVREG, 300, False),     # fresh wave tier: packed
             (abi.AM_MVREG, 5000, True),     # big view: the big-read inclusion pass
             (abi.AM_BCOUNTER, 30, True),    # rows tier (D > 8)
             (abi.AM_BCOUNTER, 3000, True),  # bounded-counter wave (D > 8)
             (abi.AM_BCOUNTER, 9000, False)]  # bounded-counter runs: packed
    kt = np.array([c[0] for c in cases], np.uint8)
    lens = np.array([c[1] for c in cases], np.uint64)
    kcols = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)  # back-to-back keys
    starts = kcols[:-1]
    cfg = dict(bench.CONFIGS["c5"], type=0)  # a mixed config at D = 16
    got = bench.lag_keys(cfg, _log(), kcols, kt, None)
    for (t, n, want), s0, g in zip(cases, starts, got):
        if t in (abi.AM_PN, abi.AM_LWW, abi.AM_MVREG) and n <= 16:
            want = int(s0) + n <= (int(s0) & ~3) + 16  # the quad test is on the aligned start
        assert bool(g) == want, (t, n, int(s0))
    # at D <= 8 the bounded-counter tiers keep the packed view
    got8 = bench.lag_keys(dict(cfg, n_dc=8), _log(), kcols, kt, None)
    assert not got8[kt == abi.AM_BCOUNTER].any()
