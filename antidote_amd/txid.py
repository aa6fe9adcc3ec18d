"""Host mirror of the TxId map (am_txid, include/antidote_mat.h): the external term format of
a #tx_id{local_start_time, server_pid} (include/antidote.hrl:192-195) -> the u64 id the device
compares for is_op_in_snapshot/7's `TxId == Op#clocksi_payload.txid`
(src/clocksi_materializer.erl:232).  Equality only: pids, ports and references are accepted,
every encoding of one term gets one id, ids are never reordered or reused."""
from __future__ import annotations

import ctypes
from typing import Any

from . import abi, etf


class TxIds:
    def __init__(self):
        self.L = abi.lib()
        self.handle = ctypes.c_void_p()
        abi.check(self.L.am_txid_create(ctypes.byref(self.handle)), "am_txid_create")

    def close(self):
        if self.handle:
            self.L.am_txid_destroy(self.handle)
            self.handle = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __len__(self):
        return int(self.L.am_txid_size(self.handle))

    def intern_encoded(self, b: bytes) -> int:
        v = ctypes.c_uint64()
        abi.check(self.L.am_txid_intern(self.handle, b, len(b), ctypes.byref(v)), "am_txid_intern")
        return int(v.value)

    def intern(self, txid: Any) -> int:
        """The id of a TxId term (etf.Pid / etf.Ref allowed)."""
        return self.intern_encoded(etf.encode(txid))

    def lookup_encoded(self, b: bytes):
        v = ctypes.c_uint64()
        rc = self.L.am_txid_lookup(self.handle, b, len(b), ctypes.byref(v))
        if rc == abi.AM_CODEC_ABSENT:
            return None
        abi.check(rc, "am_txid_lookup")
        return int(v.value)

    def forget_encoded(self, b: bytes) -> bool:
        rc = self.L.am_txid_forget(self.handle, b, len(b))
        if rc == abi.AM_CODEC_ABSENT:
            return False
        abi.check(rc, "am_txid_forget")
        return True

    def forget(self, txid: Any) -> bool:
        """Drop an ended transaction's entry (commit / abort)."""
        return self.forget_encoded(etf.encode(txid))


def canonical(b: bytes) -> bytes:
    """The canonical encoding am_txid keys on."""
    L = abi.lib()
    n = ctypes.c_uint64()
    rc = L.am_txid_canonical(b, len(b), None, 0, ctypes.byref(n))
    if rc not in (0, abi.AM_ERR_CAPACITY):
        abi.check(rc, "am_txid_canonical")
    buf = ctypes.create_string_buffer(int(n.value))
    abi.check(L.am_txid_canonical(b, len(b), buf, n.value, ctypes.byref(n)), "am_txid_canonical")
    return buf.raw[:int(n.value)]
