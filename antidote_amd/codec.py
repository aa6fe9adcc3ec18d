"""Host mirror of the term codec (am_codec, include/antidote_mat.h): Erlang terms <-> the
order-preserving u64 labels the device compares.  One Codec per partition."""
from __future__ import annotations

import ctypes
from typing import Any, List, Sequence, Tuple

import numpy as np

from . import abi, etf


class RelabelPending(Exception):
    pass


class Codec:
    def __init__(self):
        self.L = abi.lib()
        self.handle = ctypes.c_void_p()
        abi.check(self.L.am_codec_create(ctypes.byref(self.handle)), "am_codec_create")

    def close(self):
        if self.handle:
            self.L.am_codec_destroy(self.handle)
            self.handle = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __len__(self):
        return int(self.L.am_codec_size(self.handle))

    def intern_encoded(self, encs: Sequence[bytes]) -> Tuple[List[int], bool]:
        """Labels for encoded terms, and whether every label was re-spread (apply
        take_relabel()'s map to the device before using these labels)."""
        n = len(encs)
        bufs = [ctypes.create_string_buffer(e, len(e)) for e in encs]
        ptrs = (ctypes.c_void_p * max(n, 1))(*[ctypes.cast(b, ctypes.c_void_p).value for b in bufs])
        lens = np.array([len(e) for e in encs] or [0], np.uint64)
        out = np.zeros(max(n, 1), np.uint64)
        rl = ctypes.c_int(0)
        abi.check(self.L.am_codec_intern(self.handle, n, ptrs, lens.ctypes.data, out.ctypes.data, ctypes.byref(rl)),
                  "am_codec_intern")
        return [int(x) for x in out[:n]], bool(rl.value)

    def intern(self, terms: Sequence[Any]) -> Tuple[List[int], bool]:
        return self.intern_encoded([etf.encode(t) for t in terms])

    def label(self, term: Any) -> int:
        """The label of an interned term (KeyError if absent)."""
        b = etf.encode(term)
        v = ctypes.c_uint64()
        rc = self.L.am_codec_lookup(self.handle, b, len(b), ctypes.byref(v))
        if rc == abi.AM_CODEC_ABSENT:
            raise KeyError(term)
        abi.check(rc, "am_codec_lookup")
        return int(v.value)

    def encoded(self, label: int) -> bytes:
        n = ctypes.c_uint64()
        abi.check(self.L.am_codec_term(self.handle, label, None, 0, ctypes.byref(n)), "am_codec_term")
        buf = ctypes.create_string_buffer(max(int(n.value), 1))
        abi.check(self.L.am_codec_term(self.handle, label, buf, n.value, ctypes.byref(n)), "am_codec_term")
        return buf.raw[:int(n.value)]

    def term(self, label: int) -> Any:
        return etf.decode(self.encoded(label))

    def take_relabel(self) -> Tuple[np.ndarray, np.ndarray]:
        """The pending old -> new label map (old increasing); empty when none."""
        n = ctypes.c_uint64()
        abi.check(self.L.am_codec_take_relabel(self.handle, None, None, 0, ctypes.byref(n)), "am_codec_take_relabel")
        old = np.zeros(max(int(n.value), 1), np.uint64)
        new = np.zeros_like(old)
        abi.check(self.L.am_codec_take_relabel(self.handle, old.ctypes.data, new.ctypes.data, n.value,
                                               ctypes.byref(n)), "am_codec_take_relabel")
        return old[:int(n.value)], new[:int(n.value)]

    # ---- CRDT effects and values: terms <-> labels (the NIF's conversion)
    def effect(self, type_: int, eff: Any) -> Tuple[Any, bool]:
        """A downstream effect over terms -> the same effect over labels (oplog.encode_effect
        shapes).  Returns (effect, relabeled)."""
        if type_ == abi.AM_LWW:
            ts, v = eff
            (lv,), rl = self.intern([v])
            return (ts, lv), rl
        if type_ == abi.AM_MVREG:
            if eff[0] == "reset":
                labs, rl = self.intern(list(eff[1]))
                return ("reset", labs), rl
            _, v, tok, ovr = eff
            labs, rl = self.intern([v, tok] + list(ovr))
            return ("assign", labs[0], labs[1], labs[2:]), rl
        if type_ == abi.AM_AWSET:
            flat = [t for e, add, rm in eff for t in [e] + list(add) + list(rm)]
            labs, rl = self.intern(flat)
            out, i = [], 0
            for e, add, rm in eff:
                le = labs[i]
                la = labs[i + 1:i + 1 + len(add)]
                lr = labs[i + 1 + len(add):i + 1 + len(add) + len(rm)]
                i += 1 + len(add) + len(rm)
                out.append((le, la, lr))
            return sorted(out, key=lambda x: x[0]), rl  # elem order == label order
        return eff, False

    def value(self, type_: int, v: Any) -> Any:
        """A device value (HostBatch.value shapes) over labels -> the reference's state over
        terms: LWW {Ts, Value} (<<>> for the new() register), MV [{Value, Token}], AW the
        orddict [{Elem, [Token]}] (token lists in the device's order)."""
        if type_ == abi.AM_LWW:
            ts, lab, isbin = v
            return (ts, b"" if isbin else self.term(lab))
        if type_ == abi.AM_MVREG:
            return [(self.term(a), self.term(b)) for a, b in v]
        if type_ == abi.AM_AWSET:
            out: List[Any] = []
            for a, b in v:
                e, t = self.term(a), self.term(b)
                if out and out[-1][0] == e:
                    out[-1][1].append(t)
                else:
                    out.append((e, [t]))
            return [(e, ts) for e, ts in out]
        return v


def compare(a: Any, b: Any) -> int:
    """Erlang term order of two terms, by the library's comparator."""
    x, y = etf.encode(a), etf.encode(b)
    out = ctypes.c_int()
    abi.check(abi.lib().am_codec_compare(x, len(x), y, len(y), ctypes.byref(out)), "am_codec_compare")
    return int(out.value)
