"""Device-resident snapshot of a HyperGraphDB store (the bipartite CSR of DESIGN.md section 2).

Mirrors what the reference reads on the hot path:
  * HyperGraph.getIncidenceSet(h)   (C/HyperGraph.java:1415-1418)  -> ``incidence(atom)``
  * HGStore.getLink(h)              (C/HGStore.java:179-191)        -> ``targets(link)``, ``type_of(link)``
with persistent handles remapped to int32 ranks in unsigned-byte handle order
(C/handle/UUID.java:364-376; IntPersistentHandle bytes via C/storage/BAUtils.java:55-80).
C = core/src/java/org/hypergraphdb in the reference.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _lib
from ._lib import check, lib, ptr


def handle_bytes(h) -> bytes:
    """Persistent-handle bytes: UUID handles are their 16 bytes; IntPersistentHandle x is stored
    as x ^ 0x80000000 big-endian (BAUtils.writeInt), so byte order == signed int order."""
    if isinstance(h, (bytes, bytearray)):
        return bytes(h)
    if isinstance(h, int):
        return ((h ^ 0x80000000) & 0xFFFFFFFF).to_bytes(4, "big")
    raise TypeError(f"unsupported handle {h!r}")


def rank_handles(handles) -> dict:
    """Order-preserving int32 remap: rank in unsigned lexicographic byte order."""
    keyed = sorted(((handle_bytes(h), h) for h in handles), key=lambda kv: kv[0])
    ranks = {}
    for i, (_, h) in enumerate(keyed):
        if h in ranks:
            raise ValueError(f"duplicate handle {h!r}")
        ranks[h] = i
    return ranks


def _desc(num_atoms, link_atom, tgt_off, tgt_idx, link_type):
    return _lib.GraphDesc(int(num_atoms), len(link_atom), ptr(link_atom), ptr(tgt_off), ptr(tgt_idx), ptr(link_type))


def _export(h, with_targets=True):
    """D2H of the device rows (hgx_graph_export) -> (num_atoms, link_atom, tgt_off, link_type[, tgt_idx])."""
    a, m, i = C.c_int64(), C.c_int64(), C.c_int64()
    check(lib().hgx_graph_info(h, C.byref(a), C.byref(m), C.byref(i)))
    la = np.empty(m.value, np.int32)
    off = np.empty(m.value + 1, np.int64)
    ty = np.empty(m.value, np.int32)
    check(lib().hgx_graph_export(h, ptr(la), ptr(off), None, ptr(ty)))
    if not with_targets:
        return a.value, la, off, ty
    tg = np.empty(int(off[-1]), np.int32)
    check(lib().hgx_graph_export(h, None, None, ptr(tg), None))
    return a.value, la, off, ty, tg


def _handle_table(handles, num_atoms):
    if handles is None:
        return None, 0
    rows = [handle_bytes(h) for h in handles]
    if len(rows) != num_atoms:
        raise ValueError("the handle table needs one handle per atom rank")
    width = len(rows[0]) if rows else 0
    if any(len(r) != width for r in rows) or width > 64:
        raise ValueError("handles must have one byte width (<= 64)")
    return np.frombuffer(b"".join(rows), np.uint8).copy(), width


def write_snapshot(path, num_atoms, link_atom, tgt_off, tgt_idx, link_type=None, handles=None):
    """hgx_snapshot_write: the bipartite CSR (+ optional rank-ordered handle table) as a .hgcsr file."""
    la = np.ascontiguousarray(link_atom, np.int32)
    off = np.ascontiguousarray(tgt_off, np.int64)
    tg = np.ascontiguousarray(tgt_idx, np.int32)
    ty = None if link_type is None else np.ascontiguousarray(link_type, np.int32)
    if len(off) != len(la) + 1:
        raise ValueError("tgt_off must have num_links + 1 entries")
    if len(off) and int(off[-1]) != len(tg) or (ty is not None and len(ty) != len(la)):
        raise ValueError("tgt_idx / link_type sizes do not match tgt_off / link_atom")
    tab, width = _handle_table(handles, int(num_atoms))
    desc = _desc(num_atoms, la, off, tg, ty)
    check(lib().hgx_snapshot_write(os.fsencode(path), C.byref(desc), ptr(tab), width))


def read_snapshot(path) -> dict:
    """hgx_snapshot_read (checksum-verified): num_atoms, link_atom, tgt_off, tgt_idx, link_type (None
    when the file has none) and handles (uint8 [A, width] or None).  No device needed."""
    a, m, p = C.c_int64(), C.c_int64(), C.c_int64()
    hb, ht = C.c_int32(), C.c_int32()
    bpath = os.fsencode(path)
    check(lib().hgx_snapshot_info(bpath, C.byref(a), C.byref(m), C.byref(p), C.byref(hb), C.byref(ht)))
    la = np.empty(m.value, np.int32)
    off = np.empty(m.value + 1, np.int64)
    tg = np.empty(p.value, np.int32)
    ty = np.empty(m.value, np.int32)
    hs = np.empty((a.value, hb.value), np.uint8) if hb.value else None
    check(lib().hgx_snapshot_read(bpath, ptr(la), ptr(off), ptr(tg), ptr(ty), ptr(hs)))
    return {"num_atoms": a.value, "link_atom": la, "tgt_off": off, "tgt_idx": tg,
            "link_type": ty if ht.value else None, "handles": hs}


def export_store(path, handles, layouts):
    """The exporter in Python: rank the store's persistent handles, lay
    the links out as rows and write the .hgcsr file with the handle table.  ``layouts`` as in
    HyperGraphSnapshot.from_layouts.  Returns handle -> rank."""
    ranks = rank_handles(handles)
    la, off, tg, ty = _rows_from_layouts(ranks, layouts)
    by_rank = [None] * len(ranks)
    for h, r in ranks.items():
        by_rank[r] = h
    write_snapshot(path, len(ranks), la, off, tg, ty, by_rank)
    return ranks


def _rows_from_layouts(ranks, layouts):
    links = sorted(layouts, key=lambda h: ranks[h])
    link_atom = np.array([ranks[h] for h in links], np.int32)
    off = np.zeros(len(links) + 1, np.int64)
    tg = []
    types = np.zeros(len(links), np.int32)
    for r, h in enumerate(links):
        t, targets = layouts[h]
        types[r] = int(t)
        tg.extend(ranks[x] for x in targets)
        off[r + 1] = len(tg)
    return link_atom, off, np.array(tg, np.int32), types


class HyperGraphSnapshot:
    """A snapshot placed on one MI355X.  Atoms are ids 0..A-1 (rank order).  Link row r is atom
    ``link_atom[r]`` with targets ``tgt_idx[tgt_off[r]:tgt_off[r+1]]`` and type key ``link_type[r]``."""

    def __init__(self, num_atoms, link_atom, tgt_off, tgt_idx, link_type=None, device=0, keep_host=True):
        self._h = None
        link_atom = np.ascontiguousarray(link_atom, np.int32)
        tgt_off = np.ascontiguousarray(tgt_off, np.int64)
        tgt_idx = np.ascontiguousarray(tgt_idx, np.int32)
        link_type = None if link_type is None else np.ascontiguousarray(link_type, np.int32)
        if len(tgt_off) != len(link_atom) + 1:
            raise ValueError("tgt_off must have num_links + 1 entries")
        desc = _desc(num_atoms, link_atom, tgt_off, tgt_idx, link_type)
        h = C.c_void_p()
        check(lib().hgx_graph_create(C.byref(desc), int(device), C.byref(h)))
        self._attach(h, device, num_atoms, link_atom, tgt_off, tgt_idx, link_type, keep_host)

    def _attach(self, h, device, num_atoms, link_atom, tgt_off, tgt_idx, link_type, keep_host):
        self._h = h
        self.device = device
        self.A = int(num_atoms)
        self.link_atom, self.tgt_off, self.tgt_idx, self.link_type = link_atom, tgt_off, tgt_idx, link_type
        self.M = len(self.link_atom)
        a, m, i = C.c_int64(), C.c_int64(), C.c_int64()
        check(lib().hgx_graph_info(h, C.byref(a), C.byref(m), C.byref(i)))
        self.num_incidences = i.value
        self._row_of = None
        self._keep_host = keep_host
        if not keep_host:
            # large benchmark graphs: the device copy is authoritative
            self.tgt_idx = None

    # -- the snapshot on disk (.hgcsr, include/hgx.h) ------------------------------------------
    @classmethod
    def open(cls, path, device=0, keep_host=True):
        """Map a .hgcsr file (hgx_graph_open) onto ``device``.  ``keep_host`` also reads the rows
        into host arrays for targets()/type_of()."""
        h = C.c_void_p()
        check(lib().hgx_graph_open(os.fsencode(path), int(device), C.byref(h)))
        snap = cls.__new__(cls)
        snap._h = None
        try:
            if keep_host:
                f = read_snapshot(path)
                la, off, tg, ty = f["link_atom"], f["tgt_off"], f["tgt_idx"], f["link_type"]
                n = f["num_atoms"]
            else:
                n, la, off, ty = _export(h, with_targets=False)
                tg = None
        except BaseException:
            lib().hgx_graph_destroy(h)
            raise
        snap._attach(h, device, n, la, off, tg, ty, keep_host)
        return snap

    def save(self, path, handles=None):
        """Write this snapshot as .hgcsr (rows exported from the device; ``handles``: optional
        rank-ordered persistent handles stored as the handle table)."""
        n, la, off, ty, tg = _export(self.handle, with_targets=True)
        write_snapshot(path, n, la, off, tg, ty, handles)

    def update(self, add=None, remove=(), num_atoms=None):
        """Apply one batch of link events (hgx_graph_update): ``add`` = {link atom: (type key,
        [target atoms])} for HGAtomAddedEvent, ``remove`` = link atoms for HGAtomRemovedEvent,
        ``num_atoms`` = the grown rank space.  The host mirror is refreshed from the device."""
        add = add or {}
        keys = sorted(add)
        la = np.array(keys, np.int32)
        off = np.zeros(len(keys) + 1, np.int64)
        tg, ty = [], np.zeros(len(keys), np.int32)
        for r, k in enumerate(keys):
            t, targets = add[k]
            ty[r] = int(t)
            tg.extend(int(x) for x in targets)
            off[r + 1] = len(tg)
        tg = np.array(tg, np.int32)
        rm = np.ascontiguousarray(np.asarray(list(remove), np.int32))
        A = self.A if num_atoms is None else int(num_atoms)
        check(lib().hgx_graph_update(self.handle, A, len(keys), ptr(la), ptr(off), ptr(tg), ptr(ty), len(rm),
                                     ptr(rm)))
        n, la, off, ty, tg = _export(self.handle, with_targets=self._keep_host)
        self._attach(self._h, self.device, n, la, off, tg, ty, self._keep_host)

    # -- construction from reference-side objects -------------------------------------------
    @classmethod
    def from_layouts(cls, handles, layouts, device=0):
        """``handles``: every atom's persistent handle; ``layouts``: {link handle: (type_key, [target
        handles])} = the store's link records [type, value, t0..] (C/HyperGraph.java:1603-1608).
        Returns (snapshot, ranks) where ranks maps handle -> atom id."""
        ranks = rank_handles(handles)
        link_atom, off, tg, types = _rows_from_layouts(ranks, layouts)
        snap = cls(len(ranks), link_atom, off, tg, types, device=device)
        return snap, ranks

    # -- store reads -------------------------------------------------------------------------
    @property
    def handle(self):
        if self._h is None:
            raise ValueError("snapshot closed")
        return self._h

    def row_of(self, atom) -> int:
        """link row of a link atom, -1 for a node"""
        if self._row_of is None:
            self._row_of = np.full(self.A, -1, np.int32)
            self._row_of[self.link_atom] = np.arange(self.M, dtype=np.int32)
        return int(self._row_of[atom])

    def targets(self, link_atom) -> np.ndarray:
        r = self.row_of(link_atom)
        if r < 0:
            return np.empty(0, np.int32)
        return self.tgt_idx[self.tgt_off[r]:self.tgt_off[r + 1]]

    def type_of(self, link_atom) -> int:
        r = self.row_of(link_atom)
        return -1 if r < 0 else (0 if self.link_type is None else int(self.link_type[r]))

    def incidence(self, atom) -> np.ndarray:
        """HyperGraph.getIncidenceSet(atom): incident link atoms, ascending (from the device index)."""
        n = C.c_int64()
        check(lib().hgx_graph_incidence(self.handle, int(atom), None, 0, C.byref(n)))
        out = np.empty(max(n.value, 1), np.int32)
        check(lib().hgx_graph_incidence(self.handle, int(atom), ptr(out), n.value, C.byref(n)))
        return out[: n.value]

    def degree(self, atoms) -> np.ndarray:
        a = np.ascontiguousarray(np.atleast_1d(atoms), np.int32)
        out = np.empty(len(a), np.int64)
        check(lib().hgx_graph_degree(self.handle, ptr(a), len(a), ptr(out)))
        return out

    def context(self):
        """An execution context of this snapshot (hgx_graph_context): shares the device arrays, has its
        own stream, lock and scratch, so traversals on it run next to the ones on this snapshot (e.g.
        from another thread).  Store reads go to the same host mirror."""
        h = C.c_void_p()
        check(lib().hgx_graph_context(self.handle, C.byref(h)))
        ctx = type(self).__new__(type(self))
        ctx._h = None
        ctx._attach(h, self.device, self.A, self.link_atom, self.tgt_off, self.tgt_idx, self.link_type,
                    self._keep_host)
        ctx._row_of = self._row_of
        return ctx

    def set_timing(self, on=True):
        check(lib().hgx_set_timing(self.handle, 1 if on else 0))

    def set_option(self, option, value):
        check(lib().hgx_set_option(self.handle, int(option), int(value)))

    def close(self):
        if getattr(self, "_h", None) is not None:
            lib().hgx_graph_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
