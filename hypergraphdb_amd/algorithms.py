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

    def stats(self, accounting=True, raw=False):
        """Kernel timings (timing enabled), algorithmic bytes; with ``accounting`` also the
        TEPS numerator, |U_d| and the SURVEY.md 8(d) bytes (runs the accounting kernels).
        ``raw``: the hgx_bfs_stats struct itself (``.as_dict()`` later, outside a timed loop)."""
        s = _lib.BfsStats()
        check(lib().hgx_bfs_result_stats(self._h, 1 if accounting else 0, C.byref(s)))
        return s if raw else s.as_dict()

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


class SequenceResult:
    """Order-exact traversal result: per seed, the (link, atom) pairs next() returns, in order,
    with each atom's distance (host arrays)."""

    def __init__(self, handle, seeds):
        self.seeds = np.asarray(seeds, np.int32)
        try:
            ns, npairs, nl = C.c_int32(), C.c_int64(), C.c_int32()
            check(lib().hgx_seq_result_info(handle, C.byref(ns), C.byref(npairs), C.byref(nl)))
            self.n_seeds, self.n_levels = ns.value, nl.value
            self.offsets = np.zeros(self.n_seeds + 1, np.int64)
            check(lib().hgx_seq_result_offsets(handle, ptr(self.offsets)))
            n = npairs.value
            self.links = np.empty(max(n, 1), np.int32)
            self.atoms = np.empty(max(n, 1), np.int32)
            self.dists = np.empty(max(n, 1), np.int32)
            check(lib().hgx_seq_result_pairs(handle, ptr(self.links), ptr(self.atoms), ptr(self.dists)))
            self.links, self.atoms, self.dists = self.links[:n], self.atoms[:n], self.dists[:n]
            ms, tr = C.c_double(), C.c_double()
            check(lib().hgx_seq_result_stats(handle, C.byref(ms), C.byref(tr)))
            self.ms_total, self.traversed_edges = ms.value, tr.value
            nb, nl, mb, bb = C.c_int32(), C.c_int32(), C.c_double(), C.c_double()
            check(lib().hgx_seq_result_engine_stats(handle, C.byref(nb), C.byref(nl), C.byref(mb), C.byref(bb)))
            # seeds finished by the workgroup-per-seed engine / the level-synchronous reruns, and the
            # workgroup launches' device ms and algorithmic bytes
            self.n_block, self.n_level, self.ms_block, self.bytes_block = nb.value, nl.value, mb.value, bb.value
            ml, bl, pl = C.c_double(), C.c_double(), C.c_int64()
            check(lib().hgx_seq_result_level_stats(handle, C.byref(ml), C.byref(bl), C.byref(pl)))
            # the level-synchronous engine: device ms, algorithmic bytes, levels that ran as pulls
            self.ms_level, self.bytes_level, self.pull_levels = ml.value, bl.value, pl.value
            nc, mc, bc = C.c_int32(), C.c_double(), C.c_double()
            check(lib().hgx_seq_result_grid_stats(handle, C.byref(nc), C.byref(mc), C.byref(bc)))
            # the order-exact grid stage: seeds it finished, device ms, algorithmic bytes
            self.n_coop, self.ms_coop, self.bytes_coop = nc.value, mc.value, bc.value
        finally:
            lib().hgx_seq_result_free(handle)

    def pairs(self, seed_index: int):
        """(links, atoms, dists) of seed ``seed_index`` in next() order."""
        a, b = self.offsets[seed_index], self.offsets[seed_index + 1]
        return self.links[a:b], self.atoms[a:b], self.dists[a:b]


def bfs_sequence(snapshot, seeds, max_depth=None, generator: DefaultALGenerator | None = None) -> SequenceResult:
    """The exact next() sequence of HGBreadthFirstTraversal(seeds[i], generator, max_depth) for
    every i (FIFO order and discovering links as in the reference), computed on the GPU."""
    gen = generator or DefaultALGenerator(snapshot)
    opts = gen.options()
    s = np.ascontiguousarray(seeds, np.int32)
    md = _lib.HGX_UNBOUNDED if max_depth is None or max_depth >= 2**31 - 1 else int(max_depth)
    h = C.c_void_p()
    check(lib().hgx_bfs_sequence(snapshot.handle, ptr(s), len(s), md, C.byref(opts), C.byref(h)))
    return SequenceResult(h, s)


class HGBreadthFirstTraversal:
    """HGTraversal (C/algorithms/HGTraversal.java:36-63) for one start atom, backed by the GPU
    order-exact traversal: next() returns the same (link, atom) pairs in the same order as
    HGBreadthFirstTraversal.next() (:143-156), None once exhausted; isVisited(h) is true for the
    start atom and for every atom already returned (:137-141); remove() is unsupported (:98-101)."""

    def __init__(self, start, adj_list_generator: DefaultALGenerator, max_distance=None):
        self.start = int(start)
        self.gen = adj_list_generator
        self.max_distance = max_distance
        self.snapshot = adj_list_generator.graph
        self.reset()

    def reset(self):
        seq = bfs_sequence(self.snapshot, [self.start], self.max_distance, self.gen)
        self._links, self._atoms, self._dists = (x.tolist() for x in seq.pairs(0))
        self._returned = {self.start}
        self._pos = 0

    def hasNext(self):
        return self._pos < len(self._atoms)

    def next(self):
        if not self.hasNext():
            return None
        i = self._pos
        self._pos += 1
        self._returned.add(self._atoms[i])
        return (self._links[i], self._atoms[i])

    def distance(self):
        """distance of the atom returned by the last next() (the queue entry's Integer)"""
        return self._dists[self._pos - 1] if self._pos else 0

    def isVisited(self, handle):
        return int(handle) in self._returned

    def remove(self):
        raise NotImplementedError("UnsupportedOperationException")

    def __iter__(self):
        while self.hasNext():
            yield self.next()
