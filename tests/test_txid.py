"""CPU checks of the TxId map (am_txid, include/antidote_mat.h): is_op_in_snapshot/7 compares
TxIds only for equality (src/clocksi_materializer.erl:232), and #tx_id{} holds a pid
(include/antidote.hrl:192-195), which the ordered term codec refuses.  The ids must be equal
exactly when the terms are, whatever encoding of the term arrives."""
import threading

import pytest

from antidote_amd import abi, etf, txid
from antidote_amd.codec import Codec
from antidote_amd.etf import Atom, Pid, Ref

# term_to_binary(#tx_id{local_start_time = 1760000000123456, server_pid = <0.87.0>}) on node
# 'antidote@127.0.0.1' with creation 3 (OTP 23+: NEW_PID_EXT), written out byte by byte
TXID_ETF = bytes.fromhex(
    "83" "6803"                          # SMALL_TUPLE_EXT, arity 3
    "7705" "74785f6964"                  # SMALL_ATOM_UTF8_EXT 'tx_id'
    "6e0700" "40e2cfeeb54006"            # SMALL_BIG_EXT, 7 digits, positive: 1760000000123456
    "58" "7712" "616e7469646f7465403132372e302e302e31"  # NEW_PID_EXT, node 'antidote@127.0.0.1'
    "00000057" "00000000" "00000003")    # id 87, serial 0, creation 3
PID = Pid("antidote@127.0.0.1", 87, 0, 3)
TXID = (Atom("tx_id"), 1760000000123456, PID)


def test_encoder_matches_the_runtime_bytes():
    assert etf.encode(TXID) == TXID_ETF
    assert etf.decode(TXID_ETF) == TXID


def test_same_term_same_id_other_term_other_id():
    t = txid.TxIds()
    a = t.intern_encoded(TXID_ETF)
    assert t.intern(TXID) == a
    assert t.intern((Atom("tx_id"), 1760000000123457, PID)) != a
    assert t.intern((Atom("tx_id"), 1760000000123456, Pid("antidote@127.0.0.1", 88, 0, 3))) != a
    assert t.intern((Atom("tx_id"), 1760000000123456, Pid("antidote@127.0.0.2", 87, 0, 3))) != a
    assert len(t) == 4
    t.close()


def test_every_encoding_of_one_term_gets_one_id():
    t = txid.TxIds()
    a = t.intern_encoded(TXID_ETF)
    # PID_EXT (8-bit creation) and ATOM_EXT (Latin-1) spellings of the same term
    legacy = bytearray([131, 104, 3, 100, 0, 5]) + b"tx_id" + bytes.fromhex("6e070040e2cfeeb54006")
    legacy += bytes([103, 100, 0, 18]) + b"antidote@127.0.0.1" + bytes.fromhex("00000057" "00000000" "03")
    assert t.intern_encoded(bytes(legacy)) == a
    # small integers: SMALL_INTEGER_EXT / INTEGER_EXT / SMALL_BIG_EXT of 5
    five = [bytes([131, 97, 5]), bytes([131, 98, 0, 0, 0, 5]), bytes([131, 110, 1, 0, 5]),
            bytes([131, 110, 3, 0, 5, 0, 0])]
    assert len({t.intern_encoded(b) for b in five}) == 1
    # "ab" as STRING_EXT, LIST_EXT, and [97 | "b"]
    ab = [bytes([131, 107, 0, 2, 97, 98]),
          bytes([131, 108, 0, 0, 0, 2, 97, 97, 97, 98, 106]),
          bytes([131, 108, 0, 0, 0, 1, 97, 97, 107, 0, 1, 98])]
    assert len({t.intern_encoded(b) for b in ab}) == 1
    # references: NEW_REFERENCE_EXT and NEWER_REFERENCE_EXT of one ref
    r_new = etf.encode(Ref("n@h", 2, (1, 2, 3)))
    r_old = etf.encode(Ref("n@h", 2, (1, 2, 3), legacy=True))
    assert r_new != r_old and t.intern_encoded(r_new) == t.intern_encoded(r_old)
    t.close()


def test_forget_never_reuses_an_id():
    t = txid.TxIds()
    a = t.intern(TXID)
    assert t.lookup_encoded(TXID_ETF) == a
    assert t.forget(TXID)
    assert t.lookup_encoded(TXID_ETF) is None and not t.forget(TXID)
    b = t.intern(TXID)
    assert b != a and b > a
    t.close()


def test_rejects_maps_and_malformed_terms():
    t = txid.TxIds()
    with pytest.raises(abi.AmError, match="rc=-5"):
        t.intern_encoded(bytes([131, 116, 0, 0, 0, 0]))          # MAP_EXT
    with pytest.raises(abi.AmError, match="rc=-1"):
        t.intern_encoded(TXID_ETF[:-2])                            # truncated
    with pytest.raises(abi.AmError, match="rc=-1"):
        t.intern_encoded(TXID_ETF + b"\x00")                       # trailing bytes
    t.close()


def test_ordered_codec_refuses_pids_the_txid_map_accepts():
    c = Codec()
    with pytest.raises(abi.AmError):
        c.intern_encoded([TXID_ETF])
    c.close()
    t = txid.TxIds()
    assert t.intern_encoded(TXID_ETF) == 1
    t.close()


def test_concurrent_interning_is_consistent():
    t = txid.TxIds()
    terms = [(Atom("tx_id"), 1000 + i, PID) for i in range(200)]
    out = [None] * 8

    def work(k):
        out[k] = [t.intern(x) for x in (terms if k % 2 else terms[::-1])]

    th = [threading.Thread(target=work, args=(k,)) for k in range(8)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    ref = out[1]
    for k in range(8):
        assert (out[k] if k % 2 else out[k][::-1]) == ref
    assert sorted(ref) == list(range(1, 201)) and len(t) == 200
    t.close()


def test_canonical_forms_of_nested_and_improper_lists():
    # [1 | 2] keeps its improper tail; [a, {b}] re-spells the atoms as SMALL_ATOM_UTF8_EXT
    assert txid.canonical(bytes([131, 108, 0, 0, 0, 1, 97, 1, 97, 2])) == bytes.fromhex("836c0000000161016102")
    assert (txid.canonical(bytes([131, 108, 0, 0, 0, 2, 100, 0, 1, 97, 104, 1, 100, 0, 1, 98, 106]))
            == bytes.fromhex("836c0000000277016168017701626a"))
    # canonical bytes are a fixed point and decode to the same term
    c = txid.canonical(TXID_ETF)
    assert txid.canonical(c) == c and etf.decode(c) == TXID


def test_replicated_op_txids_expire_at_the_stable_snapshot():
    """Ops replicated from other DCs (inter_dc_dep_vnode -> materializer_vnode:update/2) carry
    TxIds no local coordinator ever forgets.  Their entries are stamped with the op's commit
    time {DcId, CT} and dropped once the GST covers it, so 10^5 such ops leave the map bounded
    by the ops not yet stable; a reader's held TxId stays until forget(); dropped ids are
    never handed out again."""
    t = txid.TxIds()
    remote = Pid("antidote@10.0.0.2", 40, 0, 1)
    reader = (Atom("tx_id"), 5, Pid("antidote@127.0.0.1", 90, 0, 3))
    rid = t.intern(reader)
    t.intern_op(reader, 0, 50)               # the reader's own op, committed at {0, 50}
    ids, peak = set(), 0
    n, window = 100_000, 1000
    for i in range(n):
        dc = 1 + i % 2                       # two remote DCs, CT increasing per DC
        ids.add(t.intern_op((Atom("tx_id"), 10_000 + i, remote), dc, 100 + i))
        if i % window == window - 1:         # the GST advances behind the replication stream
            t.expire({0: 0, 1: 100 + i - window // 2, 2: 100 + i - window // 2})
            peak = max(peak, len(t))
    assert len(ids) == n                     # distinct TxIds, distinct ids
    assert peak <= window + 2, peak
    assert t.lookup((Atom("tx_id"), 10_000, remote)) is None             # expired long ago
    assert t.lookup((Atom("tx_id"), 10_000 + n - 1, remote)) is not None  # not yet stable
    # the reader's entry survives a GST past its commit while held, and goes with forget()
    assert t.expire({0: 10 ** 9, 1: 0, 2: 0}) == 0 and t.lookup(reader) == rid
    assert t.forget(reader) and t.lookup(reader) is None
    # everything stable: the map empties; a re-interned TxId gets a fresh id
    t.expire({0: 10 ** 9, 1: 10 ** 9, 2: 10 ** 9})
    assert len(t) == 0
    again = t.intern_op((Atom("tx_id"), 10_000, remote), 1, 100)
    assert again not in ids and again > max(ids)
    t.close()


def test_expire_needs_the_dc_in_the_stable_snapshot():
    """A DC absent from the stable snapshot expires nothing (stable_time_functions drops DCs a
    partition lacks: no bound on them yet)."""
    t = txid.TxIds()
    t.intern_op((Atom("tx_id"), 1, PID), 3, 10)
    assert t.expire({0: 100, 1: 100}) == 0 and len(t) == 1
    assert t.expire({3: 9}) == 0 and len(t) == 1
    assert t.expire({3: 10}) == 1 and len(t) == 0
    t.close()
