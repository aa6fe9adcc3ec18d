"""The term codec (am_codec, CPU): order-preserving interning of Erlang terms into the u64
labels the device compares.

  * the comparator against the oracle's Erlang term order (oracle/ref_materializer.erl_cmp,
    the restatement of the runtime's order the CRDT rules use) on random terms;
  * labels sort exactly like their terms, decode back to the same encoding, and survive
    forced relabelling (order-preserving map, old increasing);
  * CRDT states computed over labels and decoded equal the states computed over the terms
    themselves: add-wins sets with binary elements and 20-byte binary tokens (the shape of
    test/singledc/object_log_state_SUITE.erl:95-106), MV registers with binary values, LWW
    registers with binary values and timestamp ties."""
import functools
import os
import random

import pytest

from antidote_amd import abi, etf
from antidote_amd.codec import Codec, compare
from oracle import ref_materializer as R


def _rand_term(rng, depth=0):
    k = rng.randrange(8 if depth < 2 else 4)
    if k == 0:
        return rng.choice([0, 1, 255, 256, -1, -(1 << 31), (1 << 31) - 1, 1 << 31, 1 << 70, -(1 << 70),
                           rng.randint(-10**6, 10**6), rng.randint(-(1 << 90), 1 << 90)])
    if k == 1:
        return etf.Atom(rng.choice(["a", "b", "ab", "ok", "error", "z", "increment"]))
    if k == 2:
        return bytes(rng.randrange(256) for _ in range(rng.choice([0, 1, 2, 5, 20])))
    if k == 3:
        return rng.choice([b"a", b"b", b"10", b"ab", b"", b"\x00", b"\xff"])
    if k == 4:
        return tuple(_rand_term(rng, depth + 1) for _ in range(rng.randrange(4)))
    if k == 5:
        return [_rand_term(rng, depth + 1) for _ in range(rng.randrange(4))]
    if k == 6:
        return [rng.randrange(256) for _ in range(rng.randrange(1, 5))]  # STRING_EXT
    return (rng.randint(0, 5), bytes([rng.randrange(256)]))


def _oracle_term(t):
    """etf terms -> the oracle's representation (atoms are str, binaries bytes)."""
    if isinstance(t, tuple):
        return tuple(_oracle_term(x) for x in t)
    if isinstance(t, list):
        return [_oracle_term(x) for x in t]
    if isinstance(t, etf.Atom):
        return str(t)
    return t


@pytest.mark.parametrize("seed", range(3))
def test_compare_matches_erlang_term_order(seed):
    rng = random.Random(seed)
    for _ in range(1500):
        a, b = _rand_term(rng), _rand_term(rng)
        assert compare(a, b) == R.erl_cmp(_oracle_term(a), _oracle_term(b)), (a, b)
        assert compare(a, a) == 0


def test_compare_numbers_and_special_cases():
    assert compare(1, 1.0) == 0 and compare(1, 1.5) < 0 and compare(2.5, 2) > 0
    assert compare(-(1 << 80), -1.0e20) < 0 and compare(1 << 80, 1.0e20) > 0
    assert compare(10**30, etf.Atom("a")) < 0          # number < atom
    assert compare(etf.Atom("zz"), ()) < 0              # atom < tuple
    assert compare((1, 2, 3), (9,)) > 0                 # tuples: arity first
    assert compare((9, 9), []) < 0                      # tuple < nil
    assert compare([], [0]) < 0                         # nil < list
    assert compare([1, 2], [1, 2, 0]) < 0 and compare([2], [1, 9, 9]) > 0
    assert compare([1000], b"") < 0                     # list < binary
    assert compare(b"ab", b"abc") < 0 and compare(b"b", b"abc") > 0
    assert compare([104, 105], [104, 105]) == 0 and compare(list(b"hi"), [104, 105]) == 0


def test_labels_follow_term_order_and_round_trip():
    rng = random.Random(7)
    terms = [_rand_term(rng) for _ in range(3000)] + [os.urandom(20) for _ in range(3000)]
    c = Codec()
    labels, _ = c.intern(terms)
    assert all(1 <= x <= (1 << 64) - 2 for x in labels)
    for t, lab in zip(terms, labels):
        assert c.label(t) == lab
    # equal terms share a label; distinct terms order like their labels
    uniq = {}
    for t, lab in zip(terms, labels):
        uniq.setdefault(lab, t)
    order = sorted(uniq.values(), key=functools.cmp_to_key(lambda a, b: R.erl_cmp(_oracle_term(a), _oracle_term(b))))
    assert [c.label(t) for t in order] == sorted(uniq)
    assert len(c) == len(uniq)
    for lab, t in list(uniq.items())[:500]:
        assert c.term(lab) == t
    with pytest.raises(KeyError):
        c.label(b"never interned \x00\x01")
    c.close()


def test_forced_relabel_keeps_order_and_maps_every_label():
    c = Codec()
    lo, hi = 0, 1 << 200
    labels, rl = c.intern([lo, hi])
    assert not rl
    seen = {lo: labels[0], hi: labels[1]}
    x = hi
    relabelled = False
    for _ in range(200):  # halve the gap next to 0 until the label space runs out
        x //= 2
        (lab,), rl = c.intern([x])
        if rl:
            relabelled = True
            old, new = c.take_relabel()
            assert len(old) == len(seen) and (old[1:] > old[:-1]).all() and (new[1:] > new[:-1]).all()
            m = dict(zip(old.tolist(), new.tolist()))
            seen = {t: m[v] for t, v in seen.items()}
        seen[x] = lab
        assert all(c.label(t) == v for t, v in seen.items())
    assert relabelled
    ordered = sorted(seen)
    assert [seen[t] for t in ordered] == sorted(seen.values())
    c.close()


def test_intern_refused_while_relabel_pending():
    c = Codec()
    c.intern([0, 1 << 200])
    x, rl = 1 << 200, False
    while not rl:
        x //= 2
        _, rl = c.intern([x])
    with pytest.raises(RuntimeError):
        c.intern([b"x"])
    c.take_relabel()
    c.intern([b"x"])
    c.close()


def test_unsupported_and_malformed_terms():
    c = Codec()
    for bad in (b"\x83t\x00\x00\x00\x00", b"\x83", b"\x82a\x01", b"\x83m\x00\x00\x00\x05ab"):
        with pytest.raises(RuntimeError):
            c.intern_encoded([bad])
    c.close()


def _aw_term_state(rng, n_ops):
    """Random add-wins-set downstream effects over binary elements, 20-byte tokens."""
    elems = [bytes([rng.randrange(97, 105)]) * rng.randint(1, 2) for _ in range(6)]
    live, ops = {}, []
    for _ in range(n_ops):
        e = rng.choice(elems)
        if live.get(e) and rng.random() < 0.35:
            rm = rng.sample(live[e], rng.randint(1, len(live[e])))
            live[e] = [t for t in live[e] if t not in rm]
            ops.append([(e, [], rm)])
        else:
            tok = os.urandom(20)
            live.setdefault(e, []).append(tok)
            ops.append([(e, [tok], [])])
    return ops


def test_aw_states_over_labels_equal_term_states():
    """antidote_crdt_set_aw over labels, decoded, == the same effects over the terms (element
    orddict order and each element's token list order)."""
    rng = random.Random(11)
    for _ in range(20):
        c = Codec()
        ops = _aw_term_state(rng, rng.randint(1, 60))
        st_t = []
        for eff in ops:
            st_t = R.crdt_update(R.AWSET, eff, st_t)
        lab = {}
        for eff in ops:
            for e, add, rm in eff:
                for t in [e] + add + rm:
                    if t not in lab:
                        (lab[t],), rl = c.intern([t])
                        assert not rl
        st_l = []
        for eff in ops:
            st_l = R.crdt_update(R.AWSET, [(lab[e], [lab[t] for t in a], [lab[t] for t in r]) for e, a, r in eff], st_l)
        assert [(c.term(e), [c.term(t) for t in toks]) for e, toks in st_l] == st_t
        c.close()


def test_mv_and_lww_over_labels_equal_term_states():
    rng = random.Random(12)
    c = Codec()
    for _ in range(30):
        vals = [bytes([rng.randrange(97, 100)]) for _ in range(8)]
        toks = [os.urandom(20) for _ in range(8)]
        st_t, st_l, kept = [], [], []
        for v, t in zip(vals, toks):
            ovr = rng.sample(kept, rng.randint(0, len(kept)))
            kept = [x for x in kept if x not in ovr] + [t]
            (lv, lt), _ = c.intern([v, t])
            lo = [c.label(x) for x in ovr]
            st_t = R.crdt_update(R.MVREG, (v, t, ovr), st_t)
            st_l = R.crdt_update(R.MVREG, (lv, lt, lo), st_l)
        assert [(c.term(a), c.term(b)) for a, b in st_l] == st_t
        # LWW: {Ts, Value} max with timestamp ties broken by the value's term order
        st_t = st_l = None
        for v in vals:
            ts = rng.randint(1, 3)
            lv = c.label(v)
            st_t = (ts, v) if st_t is None else R.erl_max((ts, v), st_t)
            st_l = (ts, lv) if st_l is None else R.erl_max((ts, lv), st_l)
        assert (st_l[0], c.term(st_l[1])) == st_t
    c.close()


def test_codec_symbols_exported():
    L = abi.lib()
    for name in ("am_codec_create", "am_codec_intern", "am_codec_lookup", "am_codec_term", "am_codec_take_relabel",
                 "am_codec_compare", "am_store_relabel", "am_snapcache_relabel", "am_vnode_relabel"):
        assert hasattr(L, name)
