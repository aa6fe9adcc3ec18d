"""Term codec on the device: random add-wins-set / MV-register / LWW-register histories over
real terms (binary elements and values, 20-byte binary tokens) go through am_codec into a
vnode; a forced relabel (am_codec_take_relabel -> am_vnode_relabel) is applied mid-history
to the ops cache and the snapshot cache, and every read, decoded back to terms, equals the
oracle's state computed over the terms themselves (oracle/ref_materializer.crdt_update with
Erlang term order), before and after the relabel.  A plain store relabelled in place reads
like a store built from the new labels."""
import os
import random

import pytest

from antidote_amd import abi
from antidote_amd.codec import Codec
from antidote_amd.oplog import HostLog, Op, Read
from oracle import ref_materializer as R

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mat():
    from antidote_amd.materializer import Materializer
    m = Materializer(0)
    yield m
    m.close()


class KeyHist:
    """A key's downstream effects over terms, and the oracle state after each."""

    def __init__(self, rng, t):
        self.rng, self.t, self.state = rng, t, R.crdt_new(t)
        self.elems = [bytes([97 + i]) * rng.randint(1, 3) for i in range(6)]

    def effect(self, ts):
        rng, t = self.rng, self.t
        if t == abi.AM_LWW:
            return (rng.randint(ts - 2, ts), rng.choice(self.elems))  # timestamp ties -> value order
        if t == abi.AM_MVREG:
            toks = [tok for _, tok in self.state]
            return ("assign", rng.choice(self.elems), os.urandom(20), rng.sample(toks, rng.randint(0, len(toks))))
        live = dict(self.state)
        ents = []
        for e in sorted(rng.sample(self.elems, rng.randint(1, 3))):
            if live.get(e) and rng.random() < 0.4:
                ents.append((e, [], rng.sample(live[e], rng.randint(1, len(live[e])))))
            else:
                ents.append((e, [os.urandom(20) for _ in range(rng.randint(1, 2))], []))
        return ents

    def apply(self, eff):
        if self.t == abi.AM_MVREG:
            eff = (eff[1], eff[2], eff[3])
        self.state = R.crdt_update(self.t, eff, self.state)


def _canon(t, st):
    if t == abi.AM_LWW:
        return (st[0], st[1])
    return [(a, list(b)) if t == abi.AM_AWSET else (a, b) for a, b in st]


def _force_relabel(codec, salt=0):
    """Intern integers that halve one gap until the label space there runs out."""
    x = (2 * salt + 1) << 600
    codec.intern([0, x])
    for _ in range(100000):
        x //= 2
        _, rl = codec.intern([x])
        if rl:
            return codec.take_relabel()
    raise AssertionError("no relabel")


def test_gpu_vnode_terms_with_relabel(mat):
    rng = random.Random(5)
    types = [abi.AM_AWSET, abi.AM_MVREG, abi.AM_LWW] * 4
    n = len(types)
    codec = Codec()
    vn = mat.vnode(1, n)
    hist = [KeyHist(rng, t) for t in types]
    clock = 100
    try:
        for rnd in range(8):
            batch = [[] for _ in range(n)]
            for k in range(n):
                for _ in range(rng.choice([1, 3, 12])):
                    clock += 3
                    eff = hist[k].effect(clock)
                    leff, rl = codec.effect(types[k], eff)
                    assert not rl
                    hist[k].apply(eff)
                    batch[k].append(Op(type=types[k], commit_dc=0, commit_time=clock, snap={0: clock - 1}, effect=leff))
            vn.insert(batch, types)
            hb = vn.read([Read(k, types[k], {0: clock + 1}) for k in range(n)], set_capacity=[4096] * n)
            for k in range(n):
                r = hb.result(k)
                assert r[0] == "ok", (rnd, k, r)
                assert _canon(types[k], codec.value(types[k], r[1])) == _canon(types[k], hist[k].state), (rnd, k)
            if rnd in (2, 5):
                old, new = _force_relabel(codec, rnd)
                assert len(old) > 0
                vn.relabel(old, new)
                hb = vn.read([Read(k, types[k], {0: clock + 1}) for k in range(n)], set_capacity=[4096] * n)
                for k in range(n):  # cached snapshots and ops now hold the new labels
                    r = hb.result(k)
                    assert r[0] == "ok" and _canon(types[k], codec.value(types[k], r[1])) == \
                        _canon(types[k], hist[k].state), (rnd, k, "after relabel")
    finally:
        vn.close()
        codec.close()


def test_gpu_store_relabel_equals_rebuild(mat):
    rng = random.Random(6)
    types = [abi.AM_AWSET, abi.AM_MVREG, abi.AM_LWW] * 20
    codec = Codec()
    hist = [KeyHist(rng, t) for t in types]
    effs = []
    for k in range(len(types)):  # removes / overridden tokens come from the evolving state
        es = []
        for i in range(rng.choice([2, 30, 90])):
            es.append(hist[k].effect(10 + 3 * i))
            hist[k].apply(es[-1])
        effs.append(es)

    def ops(labelled):
        return [[Op(type=types[k], commit_dc=0, commit_time=10 + 3 * i, snap={0: 9 + 3 * i}, effect=e)
                 for i, e in enumerate(labelled[k])] for k in range(len(types))]

    lab1 = [[codec.effect(types[k], e)[0] for e in es] for k, es in enumerate(effs)]
    st1 = mat.store(HostLog(1, ops(lab1), key_types=types))
    old, new = _force_relabel(codec)
    st1.relabel(old, new)
    codec_terms = [[codec.effect(types[k], e)[0] for e in es] for k, es in enumerate(effs)]  # the new labels
    st2 = mat.store(HostLog(1, ops(codec_terms), key_types=types))
    try:
        reads = [Read(k, types[k], {0: 10**6}) for k in range(len(types))]
        a = mat.read_batch(st1, reads, [4096] * len(reads))
        b = mat.read_batch(st2, reads, [4096] * len(reads))
        for k in range(len(types)):
            assert a.result(k) == b.result(k), k
            assert _canon(types[k], codec.value(types[k], a.result(k)[1])) == _canon(types[k], hist[k].state)
    finally:
        st1.close()
        st2.close()
        codec.close()
