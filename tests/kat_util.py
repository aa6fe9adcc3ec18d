"""Helpers that turn the JSON known-answer fixtures into reference-shaped terms."""
import json
import os

from oracle import ref_materializer as R

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def dc(x):
    return x


def vc(lst):
    if lst is None:
        return R.IGNORE
    return {dc(d): t for d, t in lst}


def payload(p, type_, key="abc"):
    return R.Payload(key=key, type=type_, op_param=p["param"], snapshot_time=vc(p["ss"]),
                     commit_time=(dc(p["commit"][0]), p["commit"][1]), txid=p["txid"])


def term(x):
    """JSON lists -> Erlang tuples (for the error-reason fixture)."""
    if isinstance(x, list):
        return tuple(term(e) for e in x)
    return x
