"""Synthetic op logs: parameters and the host regenerator (am_synth_host) that rebuilds
any key range of a device-generated log bit for bit (parity checks, CPU baseline)."""
from __future__ import annotations

import ctypes

import numpy as np

from . import abi
from .oplog import HostLog

SEED = 0x5EED


def params(n_keys, n_dc, type_, ops_per_key=0, seed=SEED + 2, key_base=0, max_lag=8, zipf=0.0, total_ops=0,
           hot_cap=0, universe=64, esc_ppm=0) -> abi.am_synth_params:
    p = abi.am_synth_params()
    p.seed, p.n_keys, p.ops_per_key, p.n_dc, p.type = seed, n_keys, ops_per_key, n_dc, type_
    p.key_base, p.max_lag, p.zipf_milli = key_base, max_lag, int(round(zipf * 1000))
    p.total_ops, p.hot_cap, p.universe = total_ops, hot_cap, universe
    p.esc_ppm = esc_ppm  # ops with one remote DC's entry outside the packed view (synth.h am_syn_snap_e)
    return p


def read_clock(p: abi.am_synth_params, q: float):
    c = (ctypes.c_uint64 * p.n_dc)()
    abi.check(abi.lib().am_synth_read_clock(ctypes.byref(p), q, c), "am_synth_read_clock")
    return list(c)


def host_log(p: abi.am_synth_params, k0: int, nk: int) -> HostLog:
    n_ops, n_var = ctypes.c_uint64(), ctypes.c_uint64()
    abi.check(abi.lib().am_synth_host_sizes(ctypes.byref(p), k0, nk, ctypes.byref(n_ops), ctypes.byref(n_var)),
              "am_synth_host_sizes")
    n, nv = n_ops.value, n_var.value
    has_var = p.type in (0, abi.AM_AWSET, abi.AM_MVREG, abi.AM_SYNTH_MV_BC)
    log = HostLog.__new__(HostLog)
    log.n_dc, log.n_keys, log.n_ops, log.n_var, log.has_var = p.n_dc, nk, n, nv, has_var
    log.key_off = np.zeros(nk + 1, np.uint64)
    log.key_type = np.zeros(max(nk, 1), np.uint8)
    log.key_flags = log.key_id_base = log.snap_pres = log.op_txid = log.op_id = None
    log.op_meta = np.zeros(max(n, 1), np.uint8)
    log.commit_time = np.zeros(max(n, 1), np.uint64)
    log.snap_vc = np.zeros((p.n_dc, max(n, 1)), np.uint64)
    log.p0 = np.zeros(max(n, 1), np.uint64)
    log.p1 = np.zeros(max(n, 1), np.uint64)
    log.var_off = np.zeros(n + 1, np.uint64) if has_var else None
    log.var_data = np.zeros(max(nv, 1), np.uint64) if has_var else None
    s = log.as_struct()
    s.snap_stride = log.snap_vc.shape[1]
    abi.check(abi.lib().am_synth_host(ctypes.byref(p), k0, nk, ctypes.byref(s)), "am_synth_host")
    return log
