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
        """The id of a reader's TxId term (etf.Pid / etf.Ref allowed); held until forget()."""
        return self.intern_encoded(etf.encode(txid))

    def intern_op_encoded(self, b: bytes, dc: int, ct: int) -> int:
        v = ctypes.c_uint64()
        abi.check(self.L.am_txid_intern_op(self.handle, b, len(b), dc, ct, ctypes.byref(v)), "am_txid_intern_op")
        return int(v.value)

    def intern_op(self, txid: Any, dc: int, ct: int) -> int:
        """The id of an op's TxId (#clocksi_payload.txid), stamped with the op's commit time
        {DcIndex, CT}: expire() drops it once the stable snapshot covers CT."""
        return self.intern_op_encoded(etf.encode(txid), dc, ct)

    def expire(self, stable: dict) -> int:
        """Drop the unheld op entries the stable snapshot {DcIndex: T} (the GST) covers;
        returns how many were dropped."""
        import numpy as np
        n_dc = (max(stable) + 1) if stable else 0
        vc = np.zeros(max(n_dc, 1), np.uint64)
        pres = 0
        for d, t in stable.items():
            vc[d] = t
            pres |= 1 << d
        n = ctypes.c_uint64()
        abi.check(self.L.am_txid_expire(self.handle, n_dc, vc.ctypes.data, pres, ctypes.byref(n)), "am_txid_expire")
        return int(n.value)

    def lookup_encoded(self, b: bytes):
        v = ctypes.c_uint64()
        rc = self.L.am_txid_lookup(self.handle, b, len(b), ctypes.byref(v))
        if rc == abi.AM_CODEC_ABSENT:
            return None
        abi.check(rc, "am_txid_lookup")
        return int(v.value)

    def lookup(self, txid: Any):
        """The id of a TxId term, or None when it was never interned (or forgotten / expired)."""
        return self.lookup_encoded(etf.encode(txid))

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
