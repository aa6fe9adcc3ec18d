"""ctypes view of the C ABI in include/antidote_mat.h and the loader of the in-tree
libantidote_mat.so.

torch is imported first on purpose: torch ships its own HIP runtime (SONAME
libamdhip64.so.7); loading it before libantidote_mat.so makes the library bind
to that same runtime, so torch-allocated device buffers and torch.cuda.synchronize()
interoperate with the library's stream.  torch is plumbing here (device memory,
streams, torch.distributed); every computation on the hot path is a HIP kernel
of libantidote_mat.so.  There is no CPU fallback: if the library is missing the
import fails loudly.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_float, c_int, c_int64, c_uint8, c_uint32, c_uint64, c_void_p

import torch  # noqa: F401  (must precede the HIP library, see module docstring)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("AM_LIB") or os.path.join(HERE, "libantidote_mat.so")  # AM_LIB: A/B of builds only

AM_PN, AM_LWW, AM_AWSET, AM_MVREG, AM_BCOUNTER = 1, 2, 3, 4, 5
TYPE_BY_NAME = {
    "antidote_crdt_counter_pn": AM_PN,
    "antidote_crdt_register_lww": AM_LWW,
    "antidote_crdt_set_aw": AM_AWSET,
    "antidote_crdt_register_mv": AM_MVREG,
    "antidote_crdt_counter_b": AM_BCOUNTER,
}
AM_OK = 0
AM_ERR_CORRUPTED_OPS_CACHE = 1
AM_ERR_UNEXPECTED_OPERATION = 2
AM_ERR_OVERFLOW = 3
AM_ERR_CAPACITY = 4
AM_ERR_INVALID = -1
AM_ERR_UNSUPPORTED = -5
AM_FLAG_MISSING_DC_LOGGED = 0x1
AM_META_BAD = 0x80
AM_KEY_BINARY, AM_KEY_TERM = 0, 1
AM_CODEC_ABSENT = 1
AM_KEY_MIXED_TYPES = 0x1
AM_MAX_DC = 32


def make_meta(dc: int, kind: int = 0, bad: bool = False) -> int:
    return (dc & 0x1F) | ((kind & 3) << 5) | (0x80 if bad else 0)


class am_op_log(ctypes.Structure):
    _fields_ = [
        ("n_dc", c_uint32), ("_pad", c_uint32),
        ("n_keys", c_uint64), ("n_ops", c_uint64), ("n_var", c_uint64), ("snap_stride", c_uint64),
        ("key_off", c_void_p), ("key_id_base", c_void_p), ("key_type", c_void_p), ("key_flags", c_void_p),
        ("op_meta", c_void_p), ("commit_time", c_void_p), ("snap_vc", c_void_p), ("snap_pres", c_void_p),
        ("op_txid", c_void_p), ("op_id", c_void_p), ("p0", c_void_p), ("p1", c_void_p),
        ("var_off", c_void_p), ("var_data", c_void_p),
        ("key_tbase", c_void_p), ("pk_vc", c_void_p),
        ("n_rec", c_uint64), ("rec_key_off", c_void_p), ("rec_g", c_void_p), ("grp", c_void_p),
        ("key_ngrp", c_void_p), ("key_end", c_void_p), ("rec_key_end", c_void_p), ("gmask", c_void_p),
        ("zone_vc", c_void_p), ("zone_gsum", c_void_p), ("prec", c_void_p), ("esc_rows", c_void_p),
        ("lag_ct", c_void_p), ("lag", c_void_p), ("key_lag", c_void_p),
    ]


class am_values(ctypes.Structure):
    _fields_ = [
        ("v0", c_void_p), ("v1", c_void_p), ("vflag", c_void_p),
        ("set_off", c_void_p), ("set_len", c_void_p), ("set_a", c_void_p), ("set_b", c_void_p),
    ]


class am_read_batch(ctypes.Structure):
    _fields_ = [
        ("n_reads", c_uint64), ("per_read_clock", c_uint32), ("type_hint", c_uint32),
        ("key", c_void_p), ("type", c_void_p), ("read_vc", c_void_p), ("read_pres", c_void_p),
        ("txid", c_void_p), ("txid_valid", c_void_p),
        ("base_ignore", c_void_p), ("base_vc", c_void_p), ("base_pres", c_void_p), ("base_last_op", c_void_p),
        ("base", am_values),
    ]


class am_read_result(ctypes.Structure):
    _fields_ = [
        ("status", c_void_p), ("new_last_op", c_void_p), ("last_ct", c_void_p), ("last_ct_pres", c_void_p),
        ("last_ct_ignore", c_void_p), ("is_new_ss", c_void_p), ("count", c_void_p), ("flags", c_void_p),
        ("value", am_values),
    ]


class am_synth_params(ctypes.Structure):
    _fields_ = [
        ("seed", c_uint64), ("n_keys", c_uint64), ("ops_per_key", c_uint32), ("n_dc", c_uint32),
        ("type", c_uint32), ("key_base", c_uint32), ("max_lag", c_uint32), ("zipf_milli", c_uint32),
        ("total_ops", c_uint64), ("hot_cap", c_uint32), ("universe", c_uint32), ("part_mask", c_uint64),
        ("esc_ppm", c_uint32), ("_pad2", c_uint32),
    ]


AM_SYNTH_MV_BC = 6
AM_STAT_OPS_SKIPPED = 0
AM_STAT_RECS_SKIPPED = 1
AM_STAT_GSUM_WORDS = 2
AM_ZONE_OPS = 256
AM_INDEX_NONE, AM_INDEX_ZONES, AM_INDEX_EXACT, AM_INDEX_SUMMARIES = 0, 1, 2, 3
AM_ERR_COLD_PATH = 5
AM_SNAPSHOT_THRESHOLD = 10
AM_SNAPCACHE_ABSENT = 0xFFFFFFFF
AM_GC_PRUNED_ALL = 0x1
AM_GC_TRIGGER = 0x2
AM_OPS_THRESHOLD = 50


# (name, restype, argtypes) of every exported symbol declared in include/antidote_mat.h
SIGNATURES = [
    ("am_abi_version", c_int, []),
    ("am_ctx_open", c_int, [c_int, POINTER(c_void_p)]),
    ("am_ctx_close", c_int, [c_void_p]),
    ("am_ctx_stream", c_void_p, [c_void_p]),
    ("am_ctx_sync", c_int, [c_void_p]),
    ("am_last_error", c_char_p, []),
    ("am_timer_start", c_int, [c_void_p]),
    ("am_ctx_stat", c_int, [c_void_p, c_int, c_void_p, c_int]),
    ("am_timer_stop", c_int, [c_void_p, POINTER(c_float)]),
    ("am_dev_alloc", c_int, [c_void_p, ctypes.c_size_t, POINTER(c_void_p)]),
    ("am_dev_free", c_int, [c_void_p, c_void_p]),
    ("am_memcpy_h2d", c_int, [c_void_p, c_void_p, c_void_p, ctypes.c_size_t]),
    ("am_memcpy_d2h", c_int, [c_void_p, c_void_p, c_void_p, ctypes.c_size_t]),
    ("am_store_create", c_int, [c_void_p, POINTER(am_op_log), POINTER(c_void_p)]),
    ("am_store_log", c_int, [c_void_p, POINTER(am_op_log)]),
    ("am_store_destroy", c_int, [c_void_p]),
    ("am_store_index", c_int, [c_void_p, c_void_p, c_int]),
    ("am_materialize", c_int, [c_void_p, POINTER(am_op_log), POINTER(am_read_batch), POINTER(am_read_result)]),
    ("am_materialize_host", c_int, [c_void_p, c_void_p, POINTER(am_read_batch), POINTER(am_read_result)]),
    ("am_gst_local_min", c_int, [c_void_p, c_uint32, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("am_comm_unique_id", c_int, [c_void_p]),
    ("am_comm_init", c_int, [c_void_p, c_int, c_int, c_void_p, POINTER(c_void_p)]),
    ("am_comm_destroy", c_int, [c_void_p]),
    ("am_gst_allreduce", c_int, [c_void_p, c_void_p, c_uint32]),
    ("am_gst_finalize", c_int, [c_void_p, c_uint32, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                                c_void_p]),
    ("am_gst_local_min_host", c_int, [c_uint32, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("am_gst_merge_lanes_host", c_int, [c_uint32, c_void_p, c_void_p]),
    ("am_gst_finalize_host", c_int, [c_uint32, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
    ("am_key_partition", c_uint32, [c_int64, c_uint32]),
    ("am_key_partition_bytes", c_uint32, [c_void_p, c_uint64, c_int, c_uint32]),
    ("am_chash_key", c_int, [c_void_p, c_uint64, c_void_p]),
    ("am_snapcache_create", c_int, [c_void_p, c_uint32, c_uint64, POINTER(c_void_p)]),
    ("am_snapcache_destroy", c_int, [c_void_p]),
    ("am_snapcache_read", c_int, [c_void_p, c_void_p, POINTER(am_op_log), POINTER(am_read_batch),
                                  POINTER(am_read_result)]),
    ("am_snapcache_read_host", c_int, [c_void_p, c_void_p, c_void_p, POINTER(am_read_batch),
                                       POINTER(am_read_result)]),
    ("am_snapcache_get", c_int, [c_void_p, c_void_p, c_uint64, POINTER(c_uint32), c_void_p, c_void_p, c_void_p,
                                 c_void_p, c_void_p, c_void_p]),
    ("am_snapcache_gc_threshold", c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("am_snapcache_read_gc", c_int, [c_void_p, c_void_p, POINTER(am_op_log), POINTER(am_read_batch), c_void_p,
                                     POINTER(am_read_result), c_void_p, c_void_p, c_void_p]),
    ("am_snapcache_get_value", c_int, [c_void_p, c_void_p, c_uint64, c_uint32, c_uint32, POINTER(c_uint32), c_void_p,
                                       c_void_p, c_void_p]),
    ("am_vnode_create", c_int, [c_void_p, c_uint32, c_uint64, POINTER(c_void_p)]),
    ("am_vnode_destroy", c_int, [c_void_p]),
    ("am_vnode_insert_host", c_int, [c_void_p, POINTER(am_op_log)]),
    ("am_vnode_read_host", c_int, [c_void_p, POINTER(am_read_batch), c_void_p, POINTER(am_read_result)]),
    ("am_vnode_parts", c_int, [c_void_p, POINTER(c_void_p), POINTER(c_void_p)]),
    ("am_vnode_key_info", c_int, [c_void_p, c_uint64, POINTER(c_uint64), POINTER(c_uint64), POINTER(c_uint64)]),
    ("am_vnode_stats", c_int, [c_void_p, POINTER(c_uint64), POINTER(c_uint64)]),
    ("am_store_update", c_int, [c_void_p, c_void_p, POINTER(am_op_log), c_void_p, c_void_p, c_void_p, c_void_p,
                                POINTER(c_void_p)]),
    ("am_store_reserve", c_int, [c_void_p, c_void_p, POINTER(c_void_p)]),
    ("am_store_apply", c_int, [c_void_p, c_void_p, c_uint64, c_void_p, POINTER(am_op_log), c_void_p, c_void_p, c_void_p,
                               c_void_p, POINTER(c_int)]),
    ("am_read_objects_host", c_int, [c_void_p, c_uint32, c_void_p, c_void_p, POINTER(am_read_batch),
                                     POINTER(am_read_result)]),
    ("am_read_objects_submit", c_int, [c_void_p, c_uint32, c_void_p, c_void_p, POINTER(am_read_batch),
                                       POINTER(am_read_result), POINTER(c_void_p)]),
    ("am_ticket_wait", c_int, [c_void_p]),
    ("am_codec_create", c_int, [POINTER(c_void_p)]),
    ("am_codec_destroy", c_int, [c_void_p]),
    ("am_codec_intern", c_int, [c_void_p, c_uint64, c_void_p, c_void_p, c_void_p, POINTER(c_int)]),
    ("am_codec_lookup", c_int, [c_void_p, c_char_p, c_uint64, POINTER(c_uint64)]),
    ("am_codec_term", c_int, [c_void_p, c_uint64, c_void_p, c_uint64, POINTER(c_uint64)]),
    ("am_codec_size", c_uint64, [c_void_p]),
    ("am_codec_take_relabel", c_int, [c_void_p, c_void_p, c_void_p, c_uint64, POINTER(c_uint64)]),
    ("am_codec_compare", c_int, [c_char_p, c_uint64, c_char_p, c_uint64, POINTER(c_int)]),
    ("am_txid_create", c_int, [POINTER(c_void_p)]),
    ("am_txid_destroy", c_int, [c_void_p]),
    ("am_txid_intern", c_int, [c_void_p, c_char_p, c_uint64, POINTER(c_uint64)]),
    ("am_txid_intern_op", c_int, [c_void_p, c_char_p, c_uint64, c_uint32, c_uint64, POINTER(c_uint64)]),
    ("am_txid_lookup", c_int, [c_void_p, c_char_p, c_uint64, POINTER(c_uint64)]),
    ("am_txid_expire", c_int, [c_void_p, c_uint32, c_void_p, c_uint32, POINTER(c_uint64)]),
    ("am_txid_forget", c_int, [c_void_p, c_char_p, c_uint64]),
    ("am_txid_size", c_uint64, [c_void_p]),
    ("am_txid_canonical", c_int, [c_char_p, c_uint64, c_void_p, c_uint64, POINTER(c_uint64)]),
    ("am_store_relabel", c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_uint64]),
    ("am_snapcache_relabel", c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_uint64]),
    ("am_vnode_relabel", c_int, [c_void_p, c_void_p, c_void_p, c_uint64]),
    ("am_synth_store", c_int, [c_void_p, POINTER(am_synth_params), POINTER(c_void_p)]),
    ("am_synth_read_clock", c_int, [POINTER(am_synth_params), c_double, c_void_p]),
    ("am_synth_key", c_uint64, [POINTER(am_synth_params), c_uint64]),
    ("am_synth_host_sizes", c_int, [POINTER(am_synth_params), c_uint64, c_uint64, POINTER(c_uint64),
                                    POINTER(c_uint64)]),
    ("am_synth_host", c_int, [POINTER(am_synth_params), c_uint64, c_uint64, POINTER(am_op_log)]),
]

_lib = None


class AmError(RuntimeError):
    pass


def lib():
    """Load libantidote_mat.so (built by __graft_entry__.build()).  Raises if absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise AmError(f"{LIB_PATH} missing: run __graft_entry__.build() (no CPU fallback exists)")
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.am_abi_version() != 12:
            raise AmError("ABI version mismatch")
        _lib = L
    return _lib


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = lib().am_last_error()
        raise AmError(f"{what} failed rc={rc}: {msg.decode() if msg else ''}")
