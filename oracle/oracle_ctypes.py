"""TEST INFRASTRUCTURE, NOT PRODUCT CODE.

ctypes front end of the C oracle (oracle/liboracle.so, built by oracle/Makefile).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
i64p = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")


class OgGraph(C.Structure):
    _fields_ = [("A", C.c_int64), ("M", C.c_int64),
                ("link_atom", C.c_void_p), ("tgt_off", C.c_void_p), ("tgt_idx", C.c_void_p),
                ("link_type", C.c_void_p), ("atom_row", C.c_void_p), ("inc_off", C.c_void_p),
                ("inc_atom", C.c_void_p), ("n_types", C.c_int64), ("type_off", C.c_void_p),
                ("type_atoms", C.c_void_p)]


class OgAlgen(C.Structure):
    _fields_ = [("link_type", C.c_int32), ("preceding", C.c_int32), ("succeeding", C.c_int32),
                ("reverse", C.c_int32), ("source", C.c_int32)]


def build(force: bool = False) -> str:
    so = os.path.join(_HERE, "liboracle.so")
    src = os.path.join(_HERE, "hgx_oracle.c")
    if force or not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.run(["make", "-C", _HERE, "-s"], check=True)
    return so


def lib():
    global _LIB
    if _LIB is None:
        L = C.CDLL(build())
        L.og_graph_build.argtypes = [C.POINTER(OgGraph), C.c_int64, C.c_int64, i32p, i64p, i32p, C.c_void_p]
        L.og_graph_build.restype = C.c_int
        L.og_graph_free.argtypes = [C.POINTER(OgGraph)]
        L.og_inc_size.argtypes = [C.POINTER(OgGraph), C.c_int32]
        L.og_inc_size.restype = C.c_int64
        L.og_inc_copy.argtypes = [C.POINTER(OgGraph), C.c_int32, i32p, C.c_int64]
        L.og_inc_copy.restype = C.c_int64
        L.og_generate.argtypes = [C.POINTER(OgGraph), C.POINTER(OgAlgen), C.c_int32, i32p, i32p, C.c_int64]
        L.og_generate.restype = C.c_int64
        L.og_bfs.argtypes = [C.POINTER(OgGraph), C.POINTER(OgAlgen), C.c_int32, C.c_int32,
                             i32p, i32p, i32p, C.c_int64, C.POINTER(C.c_int64)]
        L.og_bfs.restype = C.c_int64
        L.og_bfs_many.argtypes = [C.POINTER(OgGraph), C.POINTER(OgAlgen), i32p, C.c_int32, C.c_int32,
                                  C.c_int32, i64p, i64p, C.c_int32, C.c_double, C.POINTER(C.c_double)]
        L.og_bfs_many.restype = C.c_int
        L.og_ordered_link.argtypes = [i32p, C.c_int32, i32p, C.c_int32]
        L.og_ordered_link.restype = C.c_int
        for fn in (L.og_and_query, L.og_and_query_sets):
            fn.argtypes = [C.POINTER(OgGraph), C.c_int32, i32p, C.c_int32, i32p, C.c_int32, C.c_int32,
                           i32p, C.c_int64]
            fn.restype = C.c_int64
        L.og_and_query_many.argtypes = [C.POINTER(OgGraph), C.c_int32, i32p, i64p, i32p, i64p, i32p, i32p,
                                        i64p, C.POINTER(C.c_int64), C.c_int32]
        L.og_and_query_many.restype = C.c_int
        L.og_positioned.argtypes = [i32p, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32]
        L.og_positioned.restype = C.c_int
        L.og_and_query_ext.argtypes = [C.POINTER(OgGraph), C.c_int32, i32p, C.c_int32, i32p, C.c_int32, i32p,
                                       C.c_int32, i64p, i32p, C.c_int32, i32p, C.c_int64]
        L.og_and_query_ext.restype = C.c_int64
        _LIB = L
    return _LIB


def algen(link_type=-1, preceding=True, succeeding=True, reverse=False, source=False) -> OgAlgen:
    return OgAlgen(int(link_type), int(bool(preceding)), int(bool(succeeding)), int(bool(reverse)),
                   int(bool(source)))


class OracleGraph:
    """The oracle's snapshot model (see hgx_oracle.h og_graph)."""

    def __init__(self, num_atoms, link_atom, tgt_off, tgt_idx, link_type=None):
        self._keep = [np.ascontiguousarray(link_atom, np.int32), np.ascontiguousarray(tgt_off, np.int64),
                      np.ascontiguousarray(tgt_idx, np.int32)]
        self._type = None if link_type is None else np.ascontiguousarray(link_type, np.int32)
        self.g = OgGraph()
        rc = lib().og_graph_build(C.byref(self.g), int(num_atoms), len(self._keep[0]), self._keep[0],
                                  self._keep[1], self._keep[2],
                                  None if self._type is None else self._type.ctypes.data)
        if rc != 0:
            raise ValueError(f"og_graph_build failed: {rc}")
        self.A = int(num_atoms)
        self.M = len(self._keep[0])

    def __del__(self):
        if getattr(self, "g", None) is not None and _LIB is not None:
            _LIB.og_graph_free(C.byref(self.g))
            self.g = None

    def incidence(self, atom):
        n = lib().og_inc_size(C.byref(self.g), int(atom))
        out = np.empty(max(n, 1), np.int32)
        lib().og_inc_copy(C.byref(self.g), int(atom), out, n)
        return out[:n]

    def generate(self, src, opts=None):
        opts = opts or algen()
        cap = 1024
        while True:
            l = np.empty(cap, np.int32)
            a = np.empty(cap, np.int32)
            n = lib().og_generate(C.byref(self.g), C.byref(opts), int(src), l, a, cap)
            if n < 0:
                raise ValueError("bad src")
            if n <= cap:
                return list(zip(l[:n].tolist(), a[:n].tolist()))
            cap = n

    def bfs(self, seed, max_dist=-1, opts=None):
        """Returns (links, atoms, dists, traversed) in the reference FIFO order."""
        opts = opts or algen()
        cap = self.A
        l = np.empty(max(cap, 1), np.int32)
        a = np.empty(max(cap, 1), np.int32)
        d = np.empty(max(cap, 1), np.int32)
        tr = C.c_int64(0)
        n = lib().og_bfs(C.byref(self.g), C.byref(opts), int(seed), int(max_dist), l, a, d, cap, C.byref(tr))
        if n < 0:
            raise ValueError("bad seed")
        return l[:n], a[:n], d[:n], tr.value

    def bfs_levels(self, seed, max_dist=-1, opts=None):
        """Per-depth sorted visited sets [V_0={seed}, V_1, ...]."""
        _, a, d, _ = self.bfs(seed, max_dist, opts)
        nlev = int(d.max()) + 1 if len(d) else 1
        out = [np.array([seed], np.int32)]
        for k in range(1, nlev):
            out.append(np.sort(a[d == k]))
        return out

    def bfs_many(self, seeds, max_dist, max_levels, opts=None, nthreads=0, time_budget_s=0.0, timing=None):
        """Per-seed level counts [n, max_levels] and TEPS numerators.  With time_budget_s > 0 the
        traversals still running after that long stop early (bounded CPU-baseline sample); pass a
        dict as ``timing`` to receive the elapsed wall time."""
        opts = opts or algen()
        seeds = np.ascontiguousarray(seeds, np.int32)
        counts = np.zeros(len(seeds) * max_levels, np.int64)
        trav = np.zeros(len(seeds), np.int64)
        el = C.c_double(0)
        rc = lib().og_bfs_many(C.byref(self.g), C.byref(opts), seeds, len(seeds), int(max_dist),
                               int(max_levels), counts, trav, int(nthreads), float(time_budget_s), C.byref(el))
        if rc != 0:
            raise RuntimeError(f"og_bfs_many failed {rc}")
        if timing is not None:
            timing["elapsed_s"] = el.value
        return counts.reshape(len(seeds), max_levels), trav

    def and_query(self, type_=-1, incident=(), pattern=None, zigzag=True):
        inc = np.ascontiguousarray(list(incident) or [0], np.int32)
        pat = np.ascontiguousarray(list(pattern or []) or [0], np.int32)
        has = pattern is not None
        fn = lib().og_and_query if zigzag else lib().og_and_query_sets
        cap = 1024
        while True:
            out = np.empty(cap, np.int32)
            n = fn(C.byref(self.g), int(type_), inc, len(incident), pat, len(pattern or []), int(has), out, cap)
            if n < 0:
                return None if n == -1 else n
            if n <= cap:
                return out[:n]
            cap = n

    def and_query_ext(self, types=(), incident=(), positioned=(), patterns=(), arity=-1):
        """Extended And (see og_and_query_ext): positioned = [(target, lb, ub, complement)],
        patterns = [tuple of ids, -1 = anyHandle].  None = not accelerated (no anchor)."""
        ty = np.ascontiguousarray(list(types) or [0], np.int32)
        ic = np.ascontiguousarray(list(incident) or [0], np.int32)
        ps = np.ascontiguousarray([x for p in positioned for x in p] or [0], np.int32)
        po = np.zeros(len(patterns) + 1, np.int64)
        flat = []
        for r, p in enumerate(patterns):
            flat.extend(p)
            po[r + 1] = len(flat)
        pt = np.ascontiguousarray(flat or [0], np.int32)
        cap = 1024
        while True:
            out = np.empty(cap, np.int32)
            n = lib().og_and_query_ext(C.byref(self.g), len(types), ty, len(incident), ic, len(positioned), ps,
                                       len(patterns), po, pt, int(arity), out, cap)
            if n < 0:
                return None if n == -1 else n
            if n <= cap:
                return out[:n]
            cap = n

    def and_query_many(self, q_type, q_inc_off, q_inc, q_pat_off, q_pat, q_has_ordered, nthreads=0):
        n = len(q_type)
        counts = np.zeros(n, np.int64)
        cs = C.c_int64(0)
        rc = lib().og_and_query_many(C.byref(self.g), n, np.ascontiguousarray(q_type, np.int32),
                                     np.ascontiguousarray(q_inc_off, np.int64),
                                     np.ascontiguousarray(q_inc, np.int32),
                                     np.ascontiguousarray(q_pat_off, np.int64),
                                     np.ascontiguousarray(q_pat, np.int32),
                                     np.ascontiguousarray(q_has_ordered, np.int32), counts, C.byref(cs),
                                     int(nthreads))
        return counts, cs.value, rc


def positioned(targets, x, lb, ub, complement=False):
    t = np.ascontiguousarray(list(targets) or [0], np.int32)
    return bool(lib().og_positioned(t, len(targets), int(x), int(lb), int(ub), int(bool(complement))))


def ordered_link(targets, pattern):
    t = np.ascontiguousarray(list(targets) or [0], np.int32)
    p = np.ascontiguousarray(list(pattern) or [0], np.int32)
    return bool(lib().og_ordered_link(t, len(targets), p, len(pattern)))
