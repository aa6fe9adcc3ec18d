"""Host mirror of the reference's materializer interface over the HIP library.

    clocksi_materializer:materialize/4  (src/clocksi_materializer.erl:82-101)
        -> Materializer.materialize(type, txid, min_snapshot_time, response)
    materializer_vnode:read/6 batched   (src/materializer_vnode.erl:96-102)
        -> Materializer.read_batch(store, reads)
    materializer_vnode:op_insert_gc/3 + prune_ops/2 (src/materializer_vnode.erl:565-647)
        -> Store.update(new_log, prune)
    materializer_vnode:load_from_log_to_tables/2 + load_ops/2 (:288-319)
        -> Materializer.load_ops(n_dc, ops_by_key, key_types) (a Vnode)
    stable_time_functions:get_min_time/1 + meta_data_sender:update_stable/3
        -> antidote_amd.gst

Every call runs the HIP kernels of libantidote_mat.so (no CPU path exists).
"""
from __future__ import annotations

import ctypes
from typing import Any, Dict, List, Optional, Sequence, Tuple

from . import abi
from .oplog import HostBatch, HostLog, Op, Read

IGNORE = None


class Store:
    """A device-resident op log (one partition's ops cache in HBM)."""

    def __init__(self, mat: "Materializer", handle: ctypes.c_void_p, n_dc: int, owned: bool = True):
        self.mat, self.handle, self.n_dc, self.owned = mat, handle, n_dc, owned

    def device_log(self) -> abi.am_op_log:
        s = abi.am_op_log()
        abi.check(abi.lib().am_store_log(self.handle, ctypes.byref(s)), "am_store_log")
        return s

    def update(self, new_log: Optional[HostLog] = None, prune: Any = None):
        """Op-cache ingestion + GC (am_store_update): returns (new Store, gc_flags[n_keys]).

        prune: None, a SnapshotCache (its snapshot_insert_gc thresholds, computed on the
        device by am_snapcache_gc_threshold), host arrays (mask[n_keys], thr_vc[n_dc][n_keys],
        thr_pres[n_keys]), or the same as device buffers (Materializer.device_array).  new_log: ops appended per key (op_insert_gc/3), ids assigned."""
        import numpy as np
        L = self.mat.L
        n_keys = int(self.device_log().n_keys)
        bufs: List[_DevBuf] = []
        tmp_store = None
        try:
            flags = _DevBuf(self.mat, max(n_keys, 1))
            bufs.append(flags)
            mask = thr = pres = None
            if isinstance(prune, SnapshotCache):
                if prune.n_keys != n_keys:  # thresholds are laid out [d * n_keys + k] per cache key
                    raise abi.AmError(f"am_store_update: snapshot cache has {prune.n_keys} keys, "
                                      f"the store {n_keys} (rc={abi.AM_ERR_INVALID})")
                mask, thr, pres = (_DevBuf(self.mat, max(n_keys, 1)), _DevBuf(self.mat, max(n_keys, 1) * 8 * self.n_dc),
                                   _DevBuf(self.mat, max(n_keys, 1) * 4))
                bufs += [mask, thr, pres]
                abi.check(L.am_snapcache_gc_threshold(self.mat.ctx, prune.handle, mask.ptr, thr.ptr, pres.ptr),
                          "am_snapcache_gc_threshold")
            elif prune is not None and isinstance(prune[0], _DevBuf):
                mask, thr, pres = prune        # device-resident (caller-owned)
            elif prune is not None:
                m, t, pr = prune
                mask = _DevBuf.of(self.mat, np.ascontiguousarray(m, np.uint8))
                thr = _DevBuf.of(self.mat, np.ascontiguousarray(t, np.uint64))
                pres = _DevBuf.of(self.mat, np.ascontiguousarray(pr, np.uint32))
                bufs += [mask, thr, pres]
            new_dev = None
            if new_log is not None:
                tmp_store = self.mat.store(new_log)
                new_dev = tmp_store.device_log()
            h = ctypes.c_void_p()
            abi.check(L.am_store_update(self.mat.ctx, self.handle, ctypes.byref(new_dev) if new_dev is not None else None,
                                        mask.ptr if mask else None, thr.ptr if thr else None,
                                        pres.ptr if pres else None, flags.ptr, ctypes.byref(h)), "am_store_update")
            out = np.zeros(max(n_keys, 1), np.uint8)
            flags.download(out)
            return Store(self.mat, h, self.n_dc), out[:n_keys]
        finally:
            for b in bufs:
                b.free()
            if tmp_store is not None:
                tmp_store.close()

    def index(self, level: int = abi.AM_INDEX_SUMMARIES):
        """Drop and rebuild the store's zone index at `level` (am_store_index: AM_INDEX_NONE,
        _ZONES bounds only, _EXACT + exact marks, _SUMMARIES + group summaries, the default)."""
        abi.check(self.mat.L.am_store_index(self.mat.ctx, self.handle, int(level)), "am_store_index")

    def reserve(self) -> "Store":
        """A copy with room for appends per key (am_store_reserve), the layout am_store_apply
        updates in place."""
        h = ctypes.c_void_p()
        abi.check(self.mat.L.am_store_reserve(self.mat.ctx, self.handle, ctypes.byref(h)), "am_store_reserve")
        return Store(self.mat, h, self.n_dc)

    def apply(self, keys: Sequence[int], new_log: Optional[HostLog] = None, prune: Any = None):
        """In-place ingestion + GC of the touched keys only (am_store_apply).  new_log: CSR over
        the touched keys (entry i appends to keys[i]); prune: (mask[n_keys], thr_vc[n_dc][n_keys],
        thr_pres[n_keys]) host arrays or device buffers.  Returns (applied, gc_flags[len(keys)]);
        applied False: some key outgrew its room and nothing was written."""
        import numpy as np
        L = self.mat.L
        m = len(keys)
        ka = np.ascontiguousarray(keys, np.uint64)
        n_keys = int(self.device_log().n_keys)
        if m and (int(ka.max()) >= n_keys or len(np.unique(ka)) != m):
            raise abi.AmError(f"am_store_apply: touched keys must be distinct and < {n_keys} (rc={abi.AM_ERR_INVALID})")
        if new_log is not None and new_log.n_keys != m:
            raise abi.AmError(f"am_store_apply: the new-op log has {new_log.n_keys} keys for {m} touched keys "
                              f"(rc={abi.AM_ERR_INVALID})")
        bufs: List[_DevBuf] = []
        tmp_store = None
        try:
            kb = _DevBuf.of(self.mat, ka)
            flags = _DevBuf(self.mat, max(m, 1))
            bufs += [kb, flags]
            mask = thr = pres = None
            if prune is not None and isinstance(prune[0], _DevBuf):
                mask, thr, pres = prune
            elif prune is not None:
                mask, thr, pres = (_DevBuf.of(self.mat, np.ascontiguousarray(prune[0], np.uint8)),
                                   _DevBuf.of(self.mat, np.ascontiguousarray(prune[1], np.uint64)),
                                   _DevBuf.of(self.mat, np.ascontiguousarray(prune[2], np.uint32)))
                bufs += [mask, thr, pres]
            new_dev = None
            if new_log is not None:
                tmp_store = self.mat.store(new_log)
                new_dev = tmp_store.device_log()
            ap = ctypes.c_int(0)
            abi.check(L.am_store_apply(self.mat.ctx, self.handle, m, kb.ptr,
                                       ctypes.byref(new_dev) if new_dev is not None else None,
                                       mask.ptr if mask else None, thr.ptr if thr else None, pres.ptr if pres else None,
                                       flags.ptr, ctypes.byref(ap)), "am_store_apply")
            out = np.zeros(max(m, 1), np.uint8)
            flags.download(out)
            return bool(ap.value), out[:m]
        finally:
            for b in bufs:
                b.free()
            if tmp_store is not None:
                tmp_store.close()

    def relabel(self, old, new):
        """Apply a codec relabel map (Codec.take_relabel) to the store's label words in place."""
        import numpy as np
        o, n = np.ascontiguousarray(old, np.uint64), np.ascontiguousarray(new, np.uint64)
        abi.check(self.mat.L.am_store_relabel(self.mat.ctx, self.handle, o.ctypes.data, n.ctypes.data, len(o)),
                  "am_store_relabel")

    def download(self) -> Dict[str, Any]:
        """The device log's columns as numpy arrays (for parity checks); op_id is always
        filled (dense ids from key_id_base when the store keeps no explicit column)."""
        import numpy as np
        s = self.device_log()
        nk, n, nd = int(s.n_keys), int(s.n_ops), int(s.n_dc)
        stride = int(s.snap_stride) or n

        def get(ptr, count, dt):
            a = np.zeros(max(count, 1), dt)
            if ptr and count:
                abi.check(self.mat.L.am_memcpy_d2h(self.mat.ctx, a.ctypes.data, ptr, count * a.itemsize), "d2h")
            return a[:count]
        key_off = get(s.key_off, nk + 1, np.uint64)
        out = {"key_off": key_off, "key_type": get(s.key_type, nk, np.uint8),
               "key_flags": get(s.key_flags, nk, np.uint8) if s.key_flags else np.zeros(nk, np.uint8),
               "op_meta": get(s.op_meta, n, np.uint8), "commit_time": get(s.commit_time, n, np.uint64),
               "snap_vc": get(s.snap_vc, nd * stride, np.uint64).reshape(nd, stride)[:, :n] if n else np.zeros((nd, 0), np.uint64),
               "snap_pres": get(s.snap_pres, n, np.uint32) if s.snap_pres else None,
               "op_txid": get(s.op_txid, n, np.uint64) if s.op_txid else None,
               "p0": get(s.p0, n, np.uint64), "p1": get(s.p1, n, np.uint64),
               "var_off": get(s.var_off, n + 1, np.uint64) if s.var_off else None,
               "var_data": get(s.var_data, int(s.n_var), np.uint64) if s.var_off else None,
               "explicit_op_id": bool(s.op_id)}
        key_end = get(s.key_end, nk, np.uint64) if s.key_end else key_off[1:]
        if s.op_id:
            out["op_id"] = get(s.op_id, n, np.uint64)
        else:
            idb = get(s.key_id_base, nk, np.uint64) if s.key_id_base else np.ones(nk, np.uint64)
            ids = np.zeros(n, np.uint64)
            for k in range(nk):
                o0, o1 = int(key_off[k]), int(key_end[k])
                ids[o0:o1] = np.arange(o1 - o0, dtype=np.uint64) + idb[k]
            out["op_id"] = ids
        if s.key_end:  # a vnode store's room for appends: the used ops only, as a dense CSR
            sel = np.concatenate([np.arange(int(key_off[k]), int(key_end[k]), dtype=np.int64) for k in range(nk)]
                                 + [np.zeros(0, np.int64)])
            dense_off = np.zeros(nk + 1, np.uint64)
            dense_off[1:] = np.cumsum((key_end - key_off[:-1]).astype(np.uint64))
            for c in ("op_meta", "commit_time", "snap_pres", "op_txid", "p0", "p1", "op_id"):
                if out[c] is not None:
                    out[c] = out[c][sel]
            out["snap_vc"] = out["snap_vc"][:, sel]
            if out["var_off"] is not None:
                vo, vd = out["var_off"], out["var_data"]
                words = [vd[int(vo[p]):int(vo[p + 1])] for p in sel]
                lens = np.array([len(w) for w in words], np.uint64)
                out["var_off"] = np.concatenate([np.zeros(1, np.uint64), np.cumsum(lens, dtype=np.uint64)])
                out["var_data"] = np.concatenate(words + [np.zeros(0, np.uint64)]).astype(np.uint64)
            out["key_off"] = dense_off
        return out

    def close(self):
        if self.handle:
            if self.owned and self.mat.ctx:  # a closed context already released its memory
                abi.lib().am_store_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class _DevBuf:
    """A device allocation through the library's own allocator (am_dev_alloc)."""

    def __init__(self, mat: "Materializer", nbytes: int):
        self.mat, self.nbytes, self.p = mat, nbytes, ctypes.c_void_p()
        abi.check(mat.L.am_dev_alloc(mat.ctx, nbytes, ctypes.byref(self.p)), "am_dev_alloc")

    @property
    def ptr(self):
        return self.p.value

    @classmethod
    def of(cls, mat, arr):
        b = cls(mat, max(arr.nbytes, 1))
        if arr.nbytes:
            abi.check(mat.L.am_memcpy_h2d(mat.ctx, b.ptr, arr.ctypes.data, arr.nbytes), "am_memcpy_h2d")
        return b

    def download(self, arr):
        abi.check(self.mat.L.am_memcpy_d2h(self.mat.ctx, arr.ctypes.data, self.ptr, min(arr.nbytes, self.nbytes)),
                  "am_memcpy_d2h")

    def free(self):
        if self.p:
            self.mat.L.am_dev_free(self.mat.ctx, self.p)
            self.p = ctypes.c_void_p()


def _cache_snapshots(mat, sc, n_dc: int, key: int, type_: int):
    """A snapshot cache's dict for a key: [(clock, last_op_id, value)] newest first (values as
    HostBatch.value renders them), or None before the key's first read."""
    import numpy as np
    nd, cap = n_dc, abi.AM_SNAPSHOT_THRESHOLD
    n = ctypes.c_uint32()
    vc = np.zeros(cap * nd, np.uint64)
    pres = np.zeros(cap, np.uint32)
    lo = np.zeros(cap, np.int64)
    v0 = np.zeros(cap, np.int64)
    v1 = np.zeros(cap, np.uint64)
    vf = np.zeros(cap, np.uint8)
    L = mat.L
    abi.check(L.am_snapcache_get(mat.ctx, sc, key, ctypes.byref(n), vc.ctypes.data, pres.ctypes.data,
                                 lo.ctypes.data, v0.ctypes.data, v1.ctypes.data, vf.ctypes.data), "am_snapcache_get")
    if n.value == abi.AM_SNAPCACHE_ABSENT:
        return None
    out = []
    for e in range(n.value):
        clock = {d: int(vc[e * nd + d]) for d in range(nd) if (int(pres[e]) >> d) & 1}
        if type_ == abi.AM_PN:
            val: Any = int(v0[e])
        elif type_ == abi.AM_LWW:
            val = (int(v0[e:e + 1].view(np.uint64)[0]), int(v1[e]), bool(vf[e]))
        else:
            nw = ctypes.c_uint32()
            abi.check(L.am_snapcache_get_value(mat.ctx, sc, key, e, 0, ctypes.byref(nw), None, None, None),
                      "am_snapcache_get_value")
            m = max(int(nw.value), 1)
            a, b, p = np.zeros(m, np.uint64), np.zeros(m, np.uint64), np.zeros(m, np.uint8)
            abi.check(L.am_snapcache_get_value(mat.ctx, sc, key, e, m, ctypes.byref(nw), a.ctypes.data,
                                               b.ctypes.data, p.ctypes.data), "am_snapcache_get_value")
            w = int(nw.value)
            if type_ == abi.AM_BCOUNTER:
                from .oplog import bc_dicts
                val = bc_dicts([(int(a[j]), int(b[j])) for j in range(w)], nd)
            else:
                val = [(int(a[j]), int(b[j])) for j in range(w)]
        out.append((clock, int(lo[e]), val))
    return out


class SnapshotCache:
    """A partition's snapshot cache on the device: reads run materializer_vnode:internal_read/7
    (src/materializer_vnode.erl:371-376) -- base from the cache, materialize/4, write-back."""

    def __init__(self, mat: "Materializer", store: "Store", n_keys: int):
        self.mat, self.store, self.n_keys = mat, store, int(n_keys)
        self.handle = ctypes.c_void_p()
        abi.check(mat.L.am_snapcache_create(mat.ctx, store.n_dc, n_keys, ctypes.byref(self.handle)),
                  "am_snapcache_create")

    def read(self, reads: Sequence[Read], set_capacity=None) -> HostBatch:
        """internal_read/7 (ShouldGC = false) for reads of distinct keys; read.base_* are ignored.
        Per read: ('ok', Value, ...) or ('error', AM_ERR_COLD_PATH) when the log would be read."""
        hb = HostBatch(self.store.n_dc, reads, set_capacity)
        b, r = hb.structs()
        abi.check(self.mat.L.am_snapcache_read_host(self.mat.ctx, self.handle, self.store.handle, ctypes.byref(b),
                                                    ctypes.byref(r)), "am_snapcache_read_host")
        return hb

    def snapshots(self, key: int, type_: int):
        """[(clock, last_op_id, value)] newest first, or None before the key's first read."""
        return _cache_snapshots(self.mat, self.handle, self.store.n_dc, key, type_)

    def relabel(self, old, new):
        """Apply a codec relabel map to the cache (key types from the store it serves)."""
        import numpy as np
        o, n = np.ascontiguousarray(old, np.uint64), np.ascontiguousarray(new, np.uint64)
        abi.check(self.mat.L.am_snapcache_relabel(self.mat.ctx, self.handle, self.store.device_log().key_type,
                                                  o.ctypes.data, n.ctypes.data, len(o)), "am_snapcache_relabel")

    def entries(self, key: int):
        """[(clock, last_op_id, v0, v1, vflag)] newest first, or None before the key's first read."""
        import numpy as np
        nd, cap = self.store.n_dc, abi.AM_SNAPSHOT_THRESHOLD
        n = ctypes.c_uint32()
        vc = np.zeros(cap * nd, np.uint64)
        pres = np.zeros(cap, np.uint32)
        lo = np.zeros(cap, np.int64)
        v0 = np.zeros(cap, np.int64)
        v1 = np.zeros(cap, np.uint64)
        vf = np.zeros(cap, np.uint8)
        abi.check(self.mat.L.am_snapcache_get(self.mat.ctx, self.handle, key, ctypes.byref(n), vc.ctypes.data,
                                              pres.ctypes.data, lo.ctypes.data, v0.ctypes.data, v1.ctypes.data,
                                              vf.ctypes.data), "am_snapcache_get")
        if n.value == abi.AM_SNAPCACHE_ABSENT:
            return None
        out = []
        for e in range(n.value):
            clock = {d: int(vc[e * nd + d]) for d in range(nd) if (int(pres[e]) >> d) & 1}
            out.append((clock, int(lo[e]), int(v0[e]), int(v1[e]), int(vf[e])))
        return out

    def close(self):
        if self.handle:
            if self.mat.ctx:
                self.mat.L.am_snapcache_destroy(self.handle)
            self.handle = ctypes.c_void_p()


class Vnode:
    """One partition's materializer_vnode state on the device (am_vnode): the ops cache and the
    snapshot cache, driven by op_insert_gc/3 and internal_read/7 with the reference's GC
    (src/materializer_vnode.erl:371-376, 515-563, 622-647)."""

    def __init__(self, mat: "Materializer", n_dc: int, n_keys: int):
        self.mat, self.n_dc, self.n_keys = mat, n_dc, n_keys
        self.handle = ctypes.c_void_p()
        abi.check(mat.L.am_vnode_create(mat.ctx, n_dc, n_keys, ctypes.byref(self.handle)), "am_vnode_create")

    def insert(self, ops_by_key: Sequence[Sequence[Op]], key_types: Sequence[int]):
        """op_insert_gc/3 for every op (each key's ops oldest -> newest; op ids are assigned)."""
        log = HostLog(self.n_dc, ops_by_key, key_types=key_types)
        s = log.as_struct()
        abi.check(self.mat.L.am_vnode_insert_host(self.handle, ctypes.byref(s)), "am_vnode_insert_host")
        self.n_keys = max(self.n_keys, len(ops_by_key))  # keys past the key space grow it

    def read(self, reads: Sequence[Read], should_gc: Optional[Sequence[bool]] = None, set_capacity=None) -> HostBatch:
        """internal_read/7 per read (read.base_* ignored); ('error', AM_ERR_COLD_PATH) for the log path."""
        import numpy as np
        hb = HostBatch(self.n_dc, reads, set_capacity)
        b, r = hb.structs()
        sg = np.ascontiguousarray([1 if x else 0 for x in should_gc], np.uint8) if should_gc is not None else None
        abi.check(self.mat.L.am_vnode_read_host(self.handle, ctypes.byref(b), sg.ctypes.data if sg is not None else None,
                                                ctypes.byref(r)), "am_vnode_read_host")
        return hb

    def key_info(self, key: int):
        """(Length, ListLen, OpCounter) of the key's ops-cache tuple."""
        a, b, c = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        abi.check(self.mat.L.am_vnode_key_info(self.handle, key, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)),
                  "am_vnode_key_info")
        return int(a.value), int(b.value), int(c.value)

    def stats(self):
        """(whole-store rebuilds, in-place applies) of the ops cache's ingestion and GC."""
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        abi.check(self.mat.L.am_vnode_stats(self.handle, ctypes.byref(a), ctypes.byref(b)), "am_vnode_stats")
        return int(a.value), int(b.value)

    def relabel(self, old, new):
        """Apply a codec relabel map (Codec.take_relabel) to the ops cache and snapshot cache."""
        import numpy as np
        o, n = np.ascontiguousarray(old, np.uint64), np.ascontiguousarray(new, np.uint64)
        abi.check(self.mat.L.am_vnode_relabel(self.handle, o.ctypes.data, n.ctypes.data, len(o)), "am_vnode_relabel")

    def _parts(self):
        st, sc = ctypes.c_void_p(), ctypes.c_void_p()
        abi.check(self.mat.L.am_vnode_parts(self.handle, ctypes.byref(st), ctypes.byref(sc)), "am_vnode_parts")
        return st, sc

    def store(self) -> Store:
        """The ops cache as a borrowed Store: valid until the next insert or read (a read's GC can
        rebuild the store when a key outgrows its room for appends)."""
        st, _ = self._parts()
        return Store(self.mat, st, self.n_dc, owned=False)

    def op_ids(self, key: int) -> List[int]:
        """The op ids in the key's ops cache, oldest first."""
        import numpy as np
        st, _ = self._parts()
        d = abi.am_op_log()  # the vnode's store is borrowed: no Store wrapper (it would destroy it)
        abi.check(self.mat.L.am_store_log(st, ctypes.byref(d)), "am_store_log")
        L = self.mat.L
        ko = np.zeros(2, np.uint64)
        abi.check(L.am_memcpy_d2h(self.mat.ctx, ko.ctypes.data, d.key_off + key * 8, 16), "am_memcpy_d2h")
        if d.key_end:
            abi.check(L.am_memcpy_d2h(self.mat.ctx, ko[1:].ctypes.data, d.key_end + key * 8, 8), "am_memcpy_d2h")
        n = int(ko[1] - ko[0])
        if n == 0:
            return []
        if d.op_id:
            ids = np.zeros(n, np.uint64)
            abi.check(L.am_memcpy_d2h(self.mat.ctx, ids.ctypes.data, d.op_id + int(ko[0]) * 8, n * 8), "am_memcpy_d2h")
            return [int(x) for x in ids]
        base = np.ones(1, np.uint64)
        if d.key_id_base:
            abi.check(L.am_memcpy_d2h(self.mat.ctx, base.ctypes.data, d.key_id_base + key * 8, 8), "am_memcpy_d2h")
        return [int(base[0]) + i for i in range(n)]

    def snapshots(self, key: int, type_: int):
        """[(clock, last_op_id, value)] newest first, or None before the key's first read."""
        _, sc = self._parts()
        return _cache_snapshots(self.mat, sc, self.n_dc, key, type_)

    def close(self):
        if self.handle:
            if self.mat.ctx:
                self.mat.L.am_vnode_destroy(self.handle)
            self.handle = ctypes.c_void_p()


class Materializer:
    """A context on one GPU (device index = local rank)."""

    def __init__(self, device: int = 0):
        self.L = abi.lib()
        self.ctx = ctypes.c_void_p()
        abi.check(self.L.am_ctx_open(device, ctypes.byref(self.ctx)), "am_ctx_open")
        self.device = device

    def close(self):
        if self.ctx:
            self.L.am_ctx_close(self.ctx)
            self.ctx = ctypes.c_void_p()

    def sync(self):
        abi.check(self.L.am_ctx_sync(self.ctx), "am_ctx_sync")

    # ---- ops cache ----
    def store(self, log: HostLog) -> Store:
        h = ctypes.c_void_p()
        s = log.as_struct()
        abi.check(self.L.am_store_create(self.ctx, ctypes.byref(s), ctypes.byref(h)), "am_store_create")
        return Store(self, h, log.n_dc)

    def device_array(self, arr) -> "_DevBuf":
        """A caller-owned copy of a host array in HBM (free with .free())."""
        import numpy as np
        return _DevBuf.of(self, np.ascontiguousarray(arr))

    def load_ops(self, n_dc: int, ops_by_key: Sequence[Sequence[Op]], key_types) -> "Vnode":
        """load_from_log_to_tables/2 -> load_ops/2 (src/materializer_vnode.erl:288-319): every
        committed op of every key, in log order, through op_insert_gc/3 -- ids 1, 2, ... per
        key and the write-triggered GC reads (snapshots cached, ops pruned, ListLen resized)
        exactly as the reference replays its log.  Returns the partition's Vnode."""
        vn = Vnode(self, n_dc, len(ops_by_key))
        vn.insert(ops_by_key, key_types)
        return vn

    def synth_store(self, params: abi.am_synth_params) -> Store:
        h = ctypes.c_void_p()
        abi.check(self.L.am_synth_store(self.ctx, ctypes.byref(params), ctypes.byref(h)), "am_synth_store")
        return Store(self, h, params.n_dc)

    # ---- the hot path ----
    def read_batch(self, store: Store, reads: Sequence[Read], set_capacity=None) -> HostBatch:
        """materializer_vnode:read/6 -> materialize/4 for a batch of keys (host memory in/out)."""
        hb = HostBatch(store.n_dc, reads, set_capacity)
        b, r = hb.structs()
        abi.check(self.L.am_materialize_host(self.ctx, store.handle, ctypes.byref(b), ctypes.byref(r)),
                  "am_materialize_host")
        return hb

    # ---- snapshot cache (materializer_vnode snapshot_cache-P in HBM) ----
    def snapshot_cache(self, store: Store, n_keys: int) -> "SnapshotCache":
        return SnapshotCache(self, store, n_keys)

    def vnode(self, n_dc: int, n_keys: int) -> Vnode:
        return Vnode(self, n_dc, n_keys)

    def materialize(self, type_: int, txid: Optional[int], min_snapshot_time: Dict[int, int],
                    ops_newest_first: Sequence[Tuple[int, Op]], base_clock: Optional[Dict[int, int]] = None,
                    base_last_op: int = 0, base_value: Any = None, n_dc: Optional[int] = None):
        """clocksi_materializer:materialize/4 for one key, with the #snapshot_get_response{} given
        as its parts (ops list newest first, as the reference passes it)."""
        ops = [op for _, op in reversed(list(ops_newest_first))]
        ids = [i for i, _ in reversed(list(ops_newest_first))]
        for op, i in zip(ops, ids):
            op.op_id = i
        dcs = set(min_snapshot_time) | set(base_clock or {})
        for op in ops:
            dcs |= set(op.snap) | {op.commit_dc}
        nd = n_dc or (max(dcs) + 1 if dcs else 1)
        log = HostLog(nd, [ops], key_types=[type_])
        st = self.store(log)
        try:
            hb = self.read_batch(st, [Read(0, type_, dict(min_snapshot_time), txid, base_clock, base_last_op,
                                           base_value)])
            return hb.result(0)
        finally:
            st.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
