"""Erlang external term format for the host side of the boundary: what enif_term_to_binary /
enif_binary_to_term do in the NIF, for the Python mirror and its tests.

Python terms: int (any size), float, Atom (str subclass) / str as atom, tuple, list
(proper), bytes (binary), Pid / Ref (the server_pid of a #tx_id{}; only the TxId map,
am_txid, accepts them).  The codec (am_codec) interns these encodings."""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import Any, Tuple


class Atom(str):
    """An Erlang atom."""


@dataclass(frozen=True)
class Pid:
    """An Erlang pid: NEW_PID_EXT (88), or PID_EXT (103, 8-bit creation) when legacy."""
    node: str
    id: int
    serial: int
    creation: int
    legacy: bool = field(default=False, compare=False)


@dataclass(frozen=True)
class Ref:
    """An Erlang reference: NEWER_REFERENCE_EXT (90), or NEW_REFERENCE_EXT (114) when legacy."""
    node: str
    creation: int
    ids: Tuple[int, ...]
    legacy: bool = field(default=False, compare=False)


def encode(t: Any) -> bytes:
    """term_to_binary/1 (minimal encodings, as the runtime emits them)."""
    out = bytearray([131])
    _enc(t, out)
    return bytes(out)


def _enc(t: Any, out: bytearray) -> None:
    if isinstance(t, bool):
        _enc(Atom("true" if t else "false"), out)
    elif isinstance(t, int):
        if 0 <= t < 256:
            out += bytes([97, t])
        elif -(1 << 31) <= t < (1 << 31):
            out += bytes([98]) + struct.pack(">i", t)
        else:
            mag = abs(t)
            digits = mag.to_bytes((mag.bit_length() + 7) // 8, "little")
            if len(digits) < 256:
                out += bytes([110, len(digits), 1 if t < 0 else 0]) + digits
            else:
                out += bytes([111]) + struct.pack(">I", len(digits)) + bytes([1 if t < 0 else 0]) + digits
    elif isinstance(t, float):
        out += bytes([70]) + struct.pack(">d", t)
    elif isinstance(t, str):  # atoms
        b = t.encode("utf-8")
        if len(b) < 256:
            out += bytes([119, len(b)]) + b
        else:
            out += bytes([118]) + struct.pack(">H", len(b)) + b
    elif isinstance(t, tuple):
        if len(t) < 256:
            out += bytes([104, len(t)])
        else:
            out += bytes([105]) + struct.pack(">I", len(t))
        for x in t:
            _enc(x, out)
    elif isinstance(t, list):
        if not t:
            out.append(106)
        elif len(t) < 65536 and all(isinstance(x, int) and not isinstance(x, bool) and 0 <= x < 256 for x in t):
            out += bytes([107]) + struct.pack(">H", len(t)) + bytes(t)
        else:
            out += bytes([108]) + struct.pack(">I", len(t))
            for x in t:
                _enc(x, out)
            out.append(106)
    elif isinstance(t, (bytes, bytearray)):
        out += bytes([109]) + struct.pack(">I", len(t)) + bytes(t)
    elif isinstance(t, Pid):
        if t.legacy:
            out.append(103)
            _enc(Atom(t.node), out)
            out += struct.pack(">IIB", t.id, t.serial, t.creation & 0xFF)
        else:
            out.append(88)
            _enc(Atom(t.node), out)
            out += struct.pack(">III", t.id, t.serial, t.creation)
    elif isinstance(t, Ref):
        if t.legacy:
            out += bytes([114]) + struct.pack(">H", len(t.ids))
            _enc(Atom(t.node), out)
            out.append(t.creation & 0xFF)
        else:
            out += bytes([90]) + struct.pack(">H", len(t.ids))
            _enc(Atom(t.node), out)
            out += struct.pack(">I", t.creation)
        for x in t.ids:
            out += struct.pack(">I", x)
    else:
        raise TypeError(f"no external term format for {type(t)}")


def decode(b: bytes) -> Any:
    """binary_to_term/1 for the encodings above."""
    if not b or b[0] != 131:
        raise ValueError("not an external term")
    t, i = _dec(b, 1)
    if i != len(b):
        raise ValueError("trailing bytes")
    return t


def _dec(b: bytes, i: int):
    tag = b[i]
    i += 1
    if tag == 97:
        return b[i], i + 1
    if tag == 98:
        return struct.unpack(">i", b[i:i + 4])[0], i + 4
    if tag in (110, 111):
        if tag == 110:
            n, i = b[i], i + 1
        else:
            n, i = struct.unpack(">I", b[i:i + 4])[0], i + 4
        sign = b[i]
        v = int.from_bytes(b[i + 1:i + 1 + n], "little")
        return (-v if sign else v), i + 1 + n
    if tag == 70:
        return struct.unpack(">d", b[i:i + 8])[0], i + 8
    if tag in (100, 118):
        n = struct.unpack(">H", b[i:i + 2])[0]
        return Atom(b[i + 2:i + 2 + n].decode("latin-1" if tag == 100 else "utf-8")), i + 2 + n
    if tag in (115, 119):
        n = b[i]
        return Atom(b[i + 1:i + 1 + n].decode("latin-1" if tag == 115 else "utf-8")), i + 1 + n
    if tag in (104, 105):
        if tag == 104:
            n, i = b[i], i + 1
        else:
            n, i = struct.unpack(">I", b[i:i + 4])[0], i + 4
        xs = []
        for _ in range(n):
            x, i = _dec(b, i)
            xs.append(x)
        return tuple(xs), i
    if tag == 106:
        return [], i
    if tag == 107:
        n = struct.unpack(">H", b[i:i + 2])[0]
        return list(b[i + 2:i + 2 + n]), i + 2 + n
    if tag == 108:
        n = struct.unpack(">I", b[i:i + 4])[0]
        i += 4
        xs = []
        for _ in range(n):
            x, i = _dec(b, i)
            xs.append(x)
        tail, i = _dec(b, i)
        if tail != []:
            raise ValueError("improper list")
        return xs, i
    if tag == 109:
        n = struct.unpack(">I", b[i:i + 4])[0]
        return bytes(b[i + 4:i + 4 + n]), i + 4 + n
    if tag in (88, 103):
        node, i = _dec(b, i)
        if tag == 88:
            pid_id, serial, creation = struct.unpack(">III", b[i:i + 12])
            return Pid(str(node), pid_id, serial, creation), i + 12
        pid_id, serial, creation = struct.unpack(">IIB", b[i:i + 9])
        return Pid(str(node), pid_id, serial, creation, legacy=True), i + 9
    if tag in (90, 114):
        n = struct.unpack(">H", b[i:i + 2])[0]
        node, i = _dec(b, i + 2)
        if tag == 90:
            creation, i = struct.unpack(">I", b[i:i + 4])[0], i + 4
        else:
            creation, i = b[i], i + 1
        ids = struct.unpack(">" + "I" * n, b[i:i + 4 * n])
        return Ref(str(node), creation, tuple(ids), legacy=tag == 114), i + 4 * n
    raise ValueError(f"unsupported tag {tag}")
