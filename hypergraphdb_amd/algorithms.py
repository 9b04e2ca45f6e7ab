"""GPU traversal behind the reference's HGTraversal / HGALGenerator API.

Reference (C = core/src/java/org/hypergraphdb):
  * HGTraversal                (C/algorithms/HGTraversal.java:36-63)
  * HGBreadthFirstTraversal    (C/algorithms/HGBreadthFirstTraversal.java:29-164)
  * DefaultALGenerator         (C/algorithms/DefaultALGenerator.java:73-593)
  * AtomTypeCondition as link predicate (C/query/AtomTypeCondition.java:121-135)

``bfs_batch`` is the batched entry (many start atoms per launch) the GPU engine is built for.
``HGBreadthFirstTraversal`` keeps the single-seed iterator contract (hasNext/next/isVisited/
reset, remove() unsupported) on top of one batch of size 1.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import HGXError, check, lib, ptr


class HGException(RuntimeError):
    """org.hypergraphdb.HGException"""


class AtomTypeCondition:
    """hg.type(T): exact type equality (no subtypes), C/query/AtomTypeCondition.java:121-135."""

    def __init__(self, type_key: int):
        self.type = int(type_key)

    def __eq__(self, o):
        return isinstance(o, AtomTypeCondition) and o.type == self.type

    def __hash__(self):
        return hash(("type", self.type))

    def __repr__(self):
        return f"type({self.type})"


class DefaultALGenerator:
    """Adjacency-list generator configuration.  Only linkPredicate in {None, AtomTypeCondition}
    and siblingPredicate None are accelerated (any other predicate: HGXUnsupported)."""

    def __init__(self, graph, link_predicate=None, sibling_predicate=None, return_preceding=True,
                 return_succeeding=True, reverse_order=False, return_source=None):
        if return_source is None:
            # the 6-argument constructor rejects both false (DefaultALGenerator.java:451-452)
            if not return_preceding and not return_succeeding:
                raise HGException("DefaultALGenerator: attempt to construct with both returnSucceeding and "
                                  "returnPreceeding set to false.")
            return_source = False
        self.graph = graph
        self.link_predicate = link_predicate
        self.sibling_predicate = sibling_predicate
        self.return_preceding = bool(return_preceding)
        self.return_succeeding = bool(return_succeeding)
        self.reverse_order = bool(reverse_order)
        self.return_source = bool(return_source)

    def options(self) -> _lib.AlgenOpts:
        if self.sibling_predicate is not None:
            raise _lib.HGXUnsupported(_lib.HGX_E_UNSUPPORTED, "siblingPredicate is not accelerated")
        if self.link_predicate is None:
            lt = _lib.HGX_NO_TYPE
        elif isinstance(self.link_predicate, AtomTypeCondition):
            lt = self.link_predicate.type
        else:
            raise _lib.HGXUnsupported(_lib.HGX_E_UNSUPPORTED, f"link predicate {self.link_predicate!r}")
        return _lib.AlgenOpts(lt, int(self.return_preceding), int(self.return_succeeding),
                              int(self.reverse_order), int(self.return_source))


class BfsResult:
    """Per-seed, per-distance visited sets of a batched traversal (device resident)."""

    def __init__(self, snapshot, handle, seeds):
        self.snapshot = snapshot
        self._h = handle
        self.seeds = np.asarray(seeds, np.int32)
        ns, nl = C.c_int32(), C.c_int32()
        check(lib().hgx_bfs_result_info(handle, C.byref(ns), C.byref(nl)))
        self.n_seeds, self.n_levels = ns.value, nl.value
        self._counts = None

    def counts(self) -> np.ndarray:
        """[n_seeds, n_levels] |V_d| per seed (V_0 = {seed})."""
        if self._counts is None:
            out = np.zeros(self.n_seeds * self.n_levels, np.int64)
            check(lib().hgx_bfs_result_counts(self._h, ptr(out)))
            self._counts = out.reshape(self.n_seeds, self.n_levels)
        return self._counts

    def visited(self, seed_index: int, depth: int) -> np.ndarray:
        """V_depth of seed ``seed_index``: ascending atom ids."""
        n = C.c_int64()
        check(lib().hgx_bfs_result_visited(self._h, int(seed_index), int(depth), None, 0, C.byref(n)))
        out = np.empty(max(n.value, 1), np.int32)
        check(lib().hgx_bfs_result_visited(self._h, int(seed_index), int(depth), ptr(out), n.value, C.byref(n)))
        return out[: n.value]

    def levels(self, seed_index: int):
        return [self.visited(seed_index, d) for d in range(self.n_levels)]

    def depth_of(self, seed_index: int, atom: int) -> int:
        d = C.c_int32()
        check(lib().hgx_bfs_result_depth_of(self._h, int(seed_index), int(atom), C.byref(d)))
        return d.value

    def stats(self, accounting=True) -> dict:
        """Kernel timings (timing enabled), algorithmic bytes; with ``accounting`` also the
        TEPS numerator, |U_d| and the SURVEY.md 8(d) bytes (runs the accounting kernels)."""
        s = _lib.BfsStats()
        check(lib().hgx_bfs_result_stats(self._h, 1 if accounting else 0, C.byref(s)))
        return s.as_dict()

    def close(self):
        if self._h is not None:
            lib().hgx_bfs_result_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def bfs_batch(snapshot, seeds, max_depth=None, generator: DefaultALGenerator | None = None) -> BfsResult:
    """HGBreadthFirstTraversal(seeds[i], generator, max_depth) for every i, run together on the GPU."""
    gen = generator or DefaultALGenerator(snapshot)
    opts = gen.options()
    s = np.ascontiguousarray(seeds, np.int32)
    md = _lib.HGX_UNBOUNDED if max_depth is None or max_depth >= 2**31 - 1 else int(max_depth)
    h = C.c_void_p()
    check(lib().hgx_bfs_batch(snapshot.handle, ptr(s), len(s), md, C.byref(opts), C.byref(h)))
    return BfsResult(snapshot, h, s)


def _reachable(mode, tg, v, t):
    idx_v = [i for i, x in enumerate(tg) if x == v]
    idx_t = [i for i, x in enumerate(tg) if x == t]
    fv, lv, ft, lt = idx_v[0], idx_v[-1], idx_t[0], idx_t[-1]
    return {0: True, 1: lt > fv, 2: ft < fv, 3: ft < lv, 4: lt > lv}[mode]


def _mode(gen):
    P, S, R, RS = gen.return_preceding, gen.return_succeeding, gen.reverse_order, gen.return_source
    if not R:
        return 1 if not P else (2 if (not S and not RS) else 0)
    return 3 if not P else (4 if (not S and not RS) else 0)


class HGBreadthFirstTraversal:
    """HGTraversal over the GPU result for one start atom.

    next() returns (link, atom) pairs by increasing distance, like the reference; within one
    distance the atoms come in ascending handle order (the reference's FIFO order within a
    level is not reproduced -- SURVEY.md 8(f) rank 3), and ``link`` is the smallest incident
    link through which the atom is reachable from the previous level."""

    def __init__(self, start, adj_list_generator: DefaultALGenerator, max_distance=None):
        self.start = int(start)
        self.gen = adj_list_generator
        self.max_distance = max_distance
        self.snapshot = adj_list_generator.graph
        self.reset()

    def reset(self):
        self._res = bfs_batch(self.snapshot, [self.start], self.max_distance, self.gen)
        self._levels = self._res.levels(0)
        self._depth = {self.start: 0}
        for d, lv in enumerate(self._levels):
            for a in lv.tolist():
                self._depth[a] = d
        self._returned = set()
        self._queue = [(d, a) for d in range(1, len(self._levels)) for a in self._levels[d].tolist()]
        self._pos = 0

    def hasNext(self):
        return self._pos < len(self._queue)

    def next(self):
        if not self.hasNext():
            return None
        d, a = self._queue[self._pos]
        self._pos += 1
        self._returned.add(a)
        return (self._link_for(a, d), a)

    def isVisited(self, handle):
        return int(handle) in self._returned

    def remove(self):
        raise NotImplementedError("UnsupportedOperationException")

    def __iter__(self):
        while self.hasNext():
            yield self.next()

    def _link_for(self, a, d):
        snap, mode = self.snapshot, _mode(self.gen)
        lt = self.gen.link_predicate.type if isinstance(self.gen.link_predicate, AtomTypeCondition) else None
        for L in snap.incidence(a).tolist():
            if lt is not None and snap.type_of(L) != lt:
                continue
            tg = snap.targets(L).tolist()
            for v in tg:
                if v != a and self._depth.get(v) == d - 1 and _reachable(mode, tg, v, a):
                    return L
        raise HGXError(_lib.HGX_E_DEVICE, f"no discovering link for atom {a}")
