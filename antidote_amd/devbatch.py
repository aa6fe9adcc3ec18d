"""Device-resident read batches and result columns (torch allocations used as plain
HBM buffers) for am_materialize: the bench and the at-scale parity tests call the
kernels with every input already in HBM."""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import numpy as np
import torch

from . import abi


def _u64_tensor(vals, device) -> torch.Tensor:
    a = np.asarray(vals, dtype=np.uint64).view(np.int64)
    return torch.from_numpy(a.copy()).to(device)


class DeviceReads:
    """A batch of reads of keys [0, n) of a device log, all of one type, sharing one
    MinSnapshotTime (the bench's "read every key at snapshot S" step), TxId = ignore,
    base snapshot = ignore (fresh) unless set_base() is used."""

    def __init__(self, n_reads: int, n_dc: int, type_: int, clock: Sequence[int], pres: Optional[int] = None,
                 device: str = "cuda", keys: Optional[torch.Tensor] = None, set_cap: int = 96,
                 types: Optional[torch.Tensor] = None):
        """type_ = the batch's type_hint (0 = mixed: `types` gives each read's type)."""
        self.n, self.n_dc, self.type = n_reads, n_dc, type_
        dev = torch.device(device)
        self.dev = dev
        self.key = keys if keys is not None else torch.arange(n_reads, dtype=torch.int64, device=dev)
        self.types = types if types is not None else torch.full((n_reads,), type_, dtype=torch.uint8, device=dev)
        present = set(int(x) for x in torch.unique(self.types).cpu().tolist()) if type_ == 0 else {type_}
        self.read_vc = _u64_tensor(list(clock), dev)
        self.read_pres = torch.tensor([pres if pres is not None else (1 << n_dc) - 1], dtype=torch.int32, device=dev)
        self.base_ignore = None
        self.base_vc = self.base_pres = self.base_last_op = None
        self.base_v0 = self.base_v1 = self.base_vflag = None
        # results
        z = lambda dt, *s: torch.zeros(*s, dtype=dt, device=dev)  # noqa: E731
        self.status = z(torch.int32, n_reads)
        self.new_last_op = z(torch.int64, n_reads)
        self.last_ct = z(torch.int64, n_dc, n_reads)
        self.last_ct_pres = z(torch.int32, n_reads)
        self.last_ct_ignore = z(torch.uint8, n_reads)
        self.is_new_ss = z(torch.uint8, n_reads)
        self.count = z(torch.int32, n_reads)
        self.flags = z(torch.uint8, n_reads)
        self.v0 = z(torch.int64, n_reads)
        self.v1 = z(torch.int64, n_reads)
        self.vflag = z(torch.uint8, n_reads)
        self.set_off = self.set_len = self.set_a = self.set_b = None
        self.set_cap = set_cap
        # value CSR: set pairs (set_cap per read) and bounded-counter (slot, value) entries (at
        # most n_dc^2 + n_dc per read: every P and D orddict entry)
        if present & {abi.AM_AWSET, abi.AM_MVREG, abi.AM_BCOUNTER}:
            bc_cap = n_dc * n_dc + n_dc
            if abi.AM_BCOUNTER not in present:
                caps = None
                self.set_off = torch.arange(0, (n_reads + 1) * set_cap, set_cap, dtype=torch.int64, device=dev)
            else:
                caps = torch.where(self.types == abi.AM_BCOUNTER, bc_cap, set_cap).to(torch.int64)
                self.set_off = torch.zeros(n_reads + 1, dtype=torch.int64, device=dev)
                self.set_off[1:] = torch.cumsum(caps, 0)
            tot = int(self.set_off[-1].item())
            self.set_len = z(torch.int32, n_reads)
            self.set_a = z(torch.int64, max(tot, 1))
            self.set_b = z(torch.int64, max(tot, 1))

    def set_base_from(self, other: "DeviceReads"):
        """Use another batch's results as the cached base snapshots (incremental reads)."""
        self.base_ignore = other.last_ct_ignore.clone()
        self.base_vc = other.last_ct.clone()
        self.base_pres = other.last_ct_pres.clone()
        self.base_last_op = other.new_last_op.clone()
        self.base_v0 = other.v0.clone()
        self.base_v1 = other.v1.clone()
        self.base_vflag = other.vflag.clone()

    def structs(self):
        p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        b = abi.am_read_batch()
        b.n_reads, b.per_read_clock, b.type_hint = self.n, 0, self.type
        b.key, b.type, b.read_vc, b.read_pres = p(self.key), p(self.types), p(self.read_vc), p(self.read_pres)
        b.base_ignore, b.base_vc, b.base_pres, b.base_last_op = (p(self.base_ignore), p(self.base_vc),
                                                                 p(self.base_pres), p(self.base_last_op))
        b.base.v0, b.base.v1, b.base.vflag = p(self.base_v0), p(self.base_v1), p(self.base_vflag)
        r = abi.am_read_result()
        r.status, r.new_last_op, r.last_ct, r.last_ct_pres = (p(self.status), p(self.new_last_op), p(self.last_ct),
                                                              p(self.last_ct_pres))
        r.last_ct_ignore, r.is_new_ss, r.count, r.flags = (p(self.last_ct_ignore), p(self.is_new_ss), p(self.count),
                                                           p(self.flags))
        r.value.v0, r.value.v1, r.value.vflag = p(self.v0), p(self.v1), p(self.vflag)
        r.value.set_off, r.value.set_len, r.value.set_a, r.value.set_b = (p(self.set_off), p(self.set_len),
                                                                          p(self.set_a), p(self.set_b))
        self._keep = (b, r)
        return b, r

    def values(self, idx):
        """Decoded values of reads idx (host), in the oracle's rendering."""
        out = []
        nd = self.n_dc
        types = self.types.cpu().numpy()
        sl = sa = sb = so = None
        if self.set_len is not None:
            sl = self.set_len.cpu().numpy()
            sa = self.set_a.cpu().numpy().view(np.uint64)
            sb = self.set_b.cpu().numpy().view(np.uint64)
            so = self.set_off.cpu().numpy()
        v0 = self.v0.cpu().numpy()
        v1 = self.v1.cpu().numpy().view(np.uint64)
        vf = self.vflag.cpu().numpy()
        for i in idx:
            t = int(types[i])
            if t in (abi.AM_AWSET, abi.AM_MVREG):
                o = int(so[i])
                out.append([(int(sa[o + j]), int(sb[o + j])) for j in range(int(sl[i]))])
            elif t == abi.AM_BCOUNTER:
                from .oplog import bc_dicts
                o = int(so[i])
                out.append(bc_dicts([(int(sa[o + j]), int(sb[o + j])) for j in range(int(sl[i]))], nd))
            elif t == abi.AM_PN:
                out.append(int(v0[i]))
            else:
                out.append((int(v0[i:i + 1].view(np.uint64)[0]), int(v1[i]), bool(vf[i])))
        return out

    def host(self, lo: int = 0, hi: Optional[int] = None):
        """Result columns of reads [lo, hi) as numpy (u64 views where the ABI is unsigned)."""
        hi = self.n if hi is None else hi
        g = lambda t: t[..., lo:hi].cpu().numpy()  # noqa: E731
        return {
            "status": g(self.status), "new_last_op": g(self.new_last_op),
            "last_ct": g(self.last_ct).view(np.uint64), "last_ct_pres": g(self.last_ct_pres).view(np.uint32),
            "last_ct_ignore": g(self.last_ct_ignore), "is_new_ss": g(self.is_new_ss),
            "count": g(self.count).view(np.uint32), "flags": g(self.flags),
            "v0": g(self.v0), "v1": g(self.v1).view(np.uint64), "vflag": g(self.vflag),
        }


def materialize(mat, dev_log: abi.am_op_log, reads: DeviceReads):
    """Launch am_materialize (asynchronous on the context stream)."""
    b, r = reads.structs()
    abi.check(mat.L.am_materialize(mat.ctx, ctypes.byref(dev_log), ctypes.byref(b), ctypes.byref(r)),
              "am_materialize")
