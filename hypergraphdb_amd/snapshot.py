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


class HyperGraphSnapshot:
    """A snapshot placed on one MI355X.  Atoms are ids 0..A-1 (rank order).  Link row r is atom
    ``link_atom[r]`` with targets ``tgt_idx[tgt_off[r]:tgt_off[r+1]]`` and type key ``link_type[r]``."""

    def __init__(self, num_atoms, link_atom, tgt_off, tgt_idx, link_type=None, device=0, keep_host=True):
        self.A = int(num_atoms)
        self.link_atom = np.ascontiguousarray(link_atom, np.int32)
        self.tgt_off = np.ascontiguousarray(tgt_off, np.int64)
        self.tgt_idx = np.ascontiguousarray(tgt_idx, np.int32)
        self.link_type = None if link_type is None else np.ascontiguousarray(link_type, np.int32)
        self.M = len(self.link_atom)
        if len(self.tgt_off) != self.M + 1:
            raise ValueError("tgt_off must have num_links + 1 entries")
        desc = _lib.GraphDesc(self.A, self.M, ptr(self.link_atom), ptr(self.tgt_off), ptr(self.tgt_idx),
                              ptr(self.link_type))
        h = C.c_void_p()
        check(lib().hgx_graph_create(C.byref(desc), int(device), C.byref(h)))
        self._h = h
        self.device = device
        a, m, i = C.c_int64(), C.c_int64(), C.c_int64()
        check(lib().hgx_graph_info(h, C.byref(a), C.byref(m), C.byref(i)))
        self.num_incidences = i.value
        self._row_of = None
        if not keep_host:
            # large benchmark graphs: the device copy is authoritative
            self.tgt_idx = None

    # -- construction from reference-side objects -------------------------------------------
    @classmethod
    def from_layouts(cls, handles, layouts, device=0):
        """``handles``: every atom's persistent handle; ``layouts``: {link handle: (type_key, [target
        handles])} = the store's link records [type, value, t0..] (C/HyperGraph.java:1603-1608).
        Returns (snapshot, ranks) where ranks maps handle -> atom id."""
        ranks = rank_handles(handles)
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
        snap = cls(len(ranks), link_atom, off, np.array(tg, np.int32), types, device=device)
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
