"""Key -> partition for every key shape log_utilities:convert_key/1 handles
(src/log_utilities.erl:100-118): integers, binaries holding integer text (any length, signed),
other binaries and other terms through riak_core_util:chash_key (SHA-1 of
term_to_binary({<<"antidote">>, B})).  The C-ABI (am_key_partition_bytes, am_chash_key) against
the oracle restatement (oracle/ref_materializer.py convert_key, Python hashlib).  CPU only: the
partition function is host code."""
import ctypes
import random

import pytest

from antidote_amd import abi
from oracle import ref_materializer as R
from tests.kat_util import load


def _c_part(b: bytes, kind: int, n: int) -> int:
    buf = ctypes.create_string_buffer(b, max(len(b), 1))
    return int(abi.lib().am_key_partition_bytes(buf, len(b), kind, n))


def test_convert_key_kat():
    for key, exp in load("kat_vnode.json")["convert_key"]["cases"]:
        if isinstance(key, str) and key.startswith("b:"):
            b = key[2:].encode()
            assert R.convert_key(b) == exp
            assert _c_part(b, abi.AM_KEY_BINARY, 1 << 31) == exp % (1 << 31)
        else:
            assert R.convert_key(key) == exp
            assert int(abi.lib().am_key_partition(key, 1 << 31)) == exp


def test_chash_key_sha1():
    rng = random.Random(7)
    for n in [0, 1, 55, 56, 63, 64, 65, 200, 1000]:
        b = bytes(rng.randrange(256) for _ in range(n))
        out = ctypes.create_string_buffer(20)
        assert abi.lib().am_chash_key(ctypes.create_string_buffer(b, max(n, 1)), n, out) == 0
        assert out.raw == R.chash_key(b)


@pytest.mark.parametrize("n_part", [1, 7, 64, 1000, (1 << 32) - 1])
def test_key_partition_bytes(n_part):
    rng = random.Random(n_part)
    keys = [b"", b"+", b"-", b"0", b"-0", b"+17", b"-45", b"007", b" 45", b"4 5", b"1_000", b"45\n",
            str(2**200 + 12345).encode(), ("-" + str(3**150)).encode(), b"\xff\x01", "ключ".encode()]
    keys += [bytes(rng.randrange(256) for _ in range(rng.randrange(1, 40))) for _ in range(60)]
    keys += [str(rng.randrange(-10**30, 10**30)).encode() for _ in range(40)]
    for b in keys:
        assert _c_part(b, abi.AM_KEY_BINARY, n_part) == R.convert_key(b) % n_part, b
        # the same bytes as term_to_binary(Key) of a non-binary term always hash
        assert _c_part(b, abi.AM_KEY_TERM, n_part) == R.convert_key(("term",), term_bytes=b) % n_part, b
