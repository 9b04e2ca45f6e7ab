"""GPU-backed And-condition evaluation behind the reference's query API.

Reference (C = core/src/java/org/hypergraphdb):
  * HGQuery.hg DSL: hg.and / hg.type / hg.incident / hg.orderedLink / hg.anyHandle /
    hg.bfs / hg.subsumed / hg.subsumes / hg.apply(hg.targetAt)   (C/HGQuery.java:364-1823)
  * ConditionToQuery (C/query/cond2qry/ConditionToQuery.java:14-18) registered per graph with
    HGQueryConfiguration.addCompiler (C/query/HGQueryConfiguration.java:48) -- consulted before
    ToQueryMap by QueryCompile.translator (C/query/QueryCompile.java:80-87).
  * ExpressionBasedQuery.expand (C/query/cond2qry/ExpressionBasedQuery.java:689-737) flattening
    nested And and adding incident(x) for every non-ANY orderedLink target.
  * SubsumedCondition / SubsumesCondition -> BFS over HGSubsumes links
    (C/query/cond2qry/ToQueryMap.java:282-370).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import HGXUnsupported, check, lib, ptr
from .algorithms import AtomTypeCondition, DefaultALGenerator, HGException, bfs_sequence

ANY = _lib.HGX_ANY_HANDLE


class IncidentCondition:
    def __init__(self, target):
        self.target = int(target)

    def __eq__(self, o):
        return isinstance(o, IncidentCondition) and o.target == self.target

    def __hash__(self):
        return hash(("incident", self.target))

    def __repr__(self):
        return f"incident({self.target})"


class OrderedLinkCondition:
    def __init__(self, *targets):
        if len(targets) == 1 and isinstance(targets[0], (list, tuple)):
            targets = tuple(targets[0])
        self.targets = tuple(int(t) for t in targets)

    def satisfies(self, snapshot, link) -> bool:
        """C/query/OrderedLinkCondition.java:92-124 (host form, used by the API, not the batch path)."""
        if snapshot.row_of(link) < 0:
            return False
        tg = snapshot.targets(link)
        i = j = 0
        while i < len(tg) and j < len(self.targets):
            if self.targets[j] == ANY or self.targets[j] == tg[i]:
                j += 1
            i += 1
        return j == len(self.targets)

    def __repr__(self):
        return f"orderedLink{self.targets}"


class LinkCondition:
    """hg.link(targets...): the link's targets include every given target
    (C/query/LinkCondition.java:101-139); expand turns it into incident(target) for every non-ANY
    target and drops it (C/query/cond2qry/ExpressionBasedQuery.java:739-746)."""

    def __init__(self, *targets):
        if len(targets) == 1 and isinstance(targets[0], (list, tuple, set)):
            targets = tuple(targets[0])
        self.targets = tuple(int(t) for t in targets)

    def __repr__(self):
        return f"links{self.targets}"


class PositionedIncidentCondition:
    """hg.incidentAt / hg.incidentNotAt (C/query/PositionedIncidentCondition.java:123-177): the
    target sits at a position in [lower, upper] (negative = from the end), or outside it with
    ``complement``."""

    def __init__(self, target, lower, upper=None, complement=False):
        self.target, self.lower = int(target), int(lower)
        self.upper = self.lower if upper is None else int(upper)
        self.complement = bool(complement)

    def record(self):
        return (self.target, self.lower, self.upper, int(self.complement))

    def __repr__(self):
        return f"incidentAt({self.target},{self.lower},{self.upper},{self.complement})"


class ArityCondition:
    """hg.arity(k) (C/query/ArityCondition.java:49-67): the link has exactly k targets."""

    def __init__(self, arity):
        self.arity = int(arity)

    def __repr__(self):
        return f"arity({self.arity})"


class TypePlusCondition:
    """hg.typePlus(base): the atom's type is the base or one of its subtypes
    (C/query/TypePlusCondition.java:26-71); expand turns it into an Or of AtomTypeConditions
    (ExpressionBasedQuery.java:606-627).  Here it carries the resulting set of type keys."""

    def __init__(self, types):
        self.types = frozenset(int(t) for t in types)

    @classmethod
    def from_subsumption(cls, snapshot, base_type_atom, subsumes_type, key_of_atom):
        """The subtypes the way TypePlusCondition.fetchSubTypes finds them: a DefaultALGenerator
        over HGSubsumes links (preceding=False, succeeding=True) from the base -- run as one GPU
        traversal.  ``key_of_atom`` maps a type atom to the type key used in link_type."""
        from .algorithms import bfs_batch
        gen = DefaultALGenerator(snapshot, AtomTypeCondition(subsumes_type), None, False, True, False)
        r = bfs_batch(snapshot, [int(base_type_atom)], None, gen)
        atoms = [int(base_type_atom)] + [int(a) for d in range(1, r.n_levels) for a in r.visited(0, d)]
        r.close()
        return cls(key_of_atom[a] for a in atoms if a in key_of_atom)

    def __repr__(self):
        return f"typePlus{sorted(self.types)}"


class And(list):
    def __repr__(self):
        return "and(" + ", ".join(map(repr, self)) + ")"


class MapCondition:
    """hg.apply(mapping, cond)"""

    def __init__(self, mapping, cond):
        self.mapping, self.cond = mapping, cond


class TargetAt:
    """hg.targetAt(graph, i): link -> its i-th target."""

    def __init__(self, snapshot, pos):
        self.snapshot, self.pos = snapshot, int(pos)

    def __call__(self, link):
        tg = self.snapshot.targets(link)
        return int(tg[self.pos]) if self.pos < len(tg) else None


class BFSCondition:
    def __init__(self, start, link_predicate=None, return_preceding=True, return_succeeding=True,
                 reverse_order=False, max_distance=None):
        self.start = int(start)
        self.link_predicate = link_predicate
        self.flags = (return_preceding, return_succeeding, reverse_order)
        self.max_distance = max_distance


class hg:
    """The subset of HGQuery.hg on the accelerated path."""

    @staticmethod
    def type(t):
        return AtomTypeCondition(t)

    @staticmethod
    def incident(h):
        return IncidentCondition(h)

    @staticmethod
    def orderedLink(*targets):
        return OrderedLinkCondition(*targets)

    @staticmethod
    def anyHandle():
        return ANY

    @staticmethod
    def link(*targets):
        return LinkCondition(*targets)

    @staticmethod
    def incidentAt(target, lower, upper=None):
        return PositionedIncidentCondition(target, lower, upper, False)

    @staticmethod
    def incidentNotAt(target, lower, upper=None):
        return PositionedIncidentCondition(target, lower, upper, True)

    @staticmethod
    def arity(k):
        return ArityCondition(k)

    @staticmethod
    def typePlus(types):
        return types if isinstance(types, TypePlusCondition) else TypePlusCondition(types)

    @staticmethod
    def and_(*conds):
        return And(conds)

    @staticmethod
    def bfs(start, link_predicate=None, return_preceding=True, return_succeeding=True, reverse_order=False):
        return BFSCondition(start, link_predicate, return_preceding, return_succeeding, reverse_order)

    @staticmethod
    def subsumed(general, subsumes_type):
        """descendants: BFS(G) over HGSubsumes links, preceding=False, succeeding=True (ToQueryMap.java:340-370)"""
        return BFSCondition(general, AtomTypeCondition(subsumes_type), False, True, False)

    @staticmethod
    def subsumes(specific, subsumes_type):
        """ancestors: the same with reverseOrder=True (ToQueryMap.java:282-312)"""
        return BFSCondition(specific, AtomTypeCondition(subsumes_type), False, True, True)

    @staticmethod
    def apply(mapping, cond):
        return MapCondition(mapping, cond)

    @staticmethod
    def targetAt(snapshot, pos):
        return TargetAt(snapshot, pos)


def _flatten(cond, out):
    if isinstance(cond, And):
        for c in cond:
            _flatten(c, out)
    else:
        out.append(cond)
    return out


_LEAVES = (AtomTypeCondition, TypePlusCondition, IncidentCondition, LinkCondition, PositionedIncidentCondition,
           OrderedLinkCondition, ArityCondition)


def normalize(cond):
    """The accelerated And shapes after ExpressionBasedQuery.expand + toDNF, as a dict
    {types (sorted list, [] = no type condition), inc, pos [(target, lb, ub, complement)],
    patterns [tuple], arity (-1 = none)} -- or "empty" when the conjunction can match nothing
    (two different exact types, two different arities).  Any other shape raises HGXUnsupported
    (a Java shim delegates those to AndToQuery)."""
    if isinstance(cond, _LEAVES):
        cond = And([cond])
    if not isinstance(cond, And):
        raise HGXUnsupported(_lib.HGX_E_UNSUPPORTED, f"not an And: {cond!r}")
    subs = _flatten(cond, [])
    if not all(isinstance(c, _LEAVES) for c in subs):
        raise HGXUnsupported(_lib.HGX_E_UNSUPPORTED, f"shape not accelerated: {cond!r}")
    tset = None
    for c in subs:   # every type condition must hold: intersect their type sets
        if isinstance(c, AtomTypeCondition):
            tset = {c.type} if tset is None else tset & {c.type}
        elif isinstance(c, TypePlusCondition):
            tset = set(c.types) if tset is None else tset & set(c.types)
    arities = {c.arity for c in subs if isinstance(c, ArityCondition)}
    if (tset is not None and not tset) or len(arities) > 1:
        return "empty"
    inc = [c.target for c in subs if isinstance(c, IncidentCondition)]
    for c in subs:
        if isinstance(c, LinkCondition):
            inc.extend(t for t in c.targets if t != ANY)
    return {"types": sorted(tset) if tset is not None else [], "inc": inc,
            "pos": [c.record() for c in subs if isinstance(c, PositionedIncidentCondition)],
            "patterns": [c.targets for c in subs if isinstance(c, OrderedLinkCondition)],
            "arity": arities.pop() if arities else -1}


def _from_tuple(q):
    """legacy (type, incident, pattern-or-None) -> the normalised dict"""
    t, inc, pat = q
    return {"types": [] if t is None or t < 0 else [int(t)], "inc": list(inc), "pos": [],
            "patterns": [] if pat is None else [tuple(pat)], "arity": -1}


class QueryResult:
    def __init__(self, offsets, ids, ms=None):
        self.offsets, self.ids, self.ms = offsets, ids, ms

    def __len__(self):
        return len(self.offsets) - 1

    def __getitem__(self, q):
        return self.ids[self.offsets[q]:self.offsets[q + 1]]


def _read_result(h, n) -> QueryResult:
    try:
        off = np.empty(n + 1, np.int64)
        check(lib().hgx_query_result_offsets(h, ptr(off)))
        ids = np.empty(max(int(off[-1]), 1), np.int32)
        check(lib().hgx_query_result_ids(h, ptr(ids)))
        a, b, c = C.c_double(), C.c_double(), C.c_double()
        check(lib().hgx_query_result_ms(h, C.byref(a), C.byref(b), C.byref(c)))
    finally:
        lib().hgx_query_result_free(h)
    return QueryResult(off, ids[: int(off[-1])], {"ms_total": a.value, "ms_match": b.value, "bytes_match": c.value})


class QuerySet:
    """A packed batch resident in device memory (hgx_query_set_create): uploaded once, run many times
    (``run(snapshot)``) without moving the queries again -- a fixed set of compiled queries re-executed
    by an application (TC/query/QueryCompilation.java:76-122)."""

    def __init__(self, snapshot, q_type, inc_off, inc, has_ordered, pat_off, pat):
        self._h = None
        arrs = [np.ascontiguousarray(q_type, np.int32), np.ascontiguousarray(inc_off, np.int64),
                np.ascontiguousarray(inc, np.int32), np.ascontiguousarray(has_ordered, np.int32),
                np.ascontiguousarray(pat_off, np.int64), np.ascontiguousarray(pat, np.int32)]
        self.n = len(arrs[0])
        h = C.c_void_p()
        check(lib().hgx_query_set_create(snapshot.handle, self.n, *(a.ctypes.data for a in arrs), C.byref(h)))
        self._h = h

    def run(self, snapshot) -> QueryResult:
        """hgx_pattern_batch_set on ``snapshot`` (or an execution context of it)."""
        h = C.c_void_p()
        check(lib().hgx_pattern_batch_set(snapshot.handle, self._h, C.byref(h)))
        return _read_result(h, self.n)

    def run_into(self, snapshot, offsets: np.ndarray, ids: np.ndarray, timing: np.ndarray | None = None) -> int:
        """hgx_pattern_batch_set_into: the results into caller arrays (``offsets``: int64[n + 1],
        ``ids``: int32); returns the number of hits.  ``ids`` holds them only when that number fits
        (``offsets`` is always filled, so a caller can size ``ids`` and run again).  ``timing``
        (float64[3], optional): device ms of the batch, ms and algorithmic bytes of the match kernel."""
        if timing is not None and (timing.dtype != np.float64 or timing.size < 3 or not timing.flags.c_contiguous):
            raise ValueError("timing must be a contiguous float64 array of 3 entries")
        if offsets.dtype != np.int64 or offsets.size < self.n + 1 or not offsets.flags.c_contiguous:
            raise ValueError(f"offsets must be a contiguous int64 array of at least {self.n + 1} entries")
        if ids.dtype != np.int32 or not ids.flags.c_contiguous:
            raise ValueError("ids must be a contiguous int32 array")
        n_ids = C.c_int64()
        check(lib().hgx_pattern_batch_set_into(snapshot.handle, self._h, offsets.ctypes.data, ids.ctypes.data,
                                               ids.size, C.byref(n_ids),
                                               None if timing is None else timing.ctypes.data))
        return n_ids.value

    def close(self):
        if self._h is not None:
            lib().hgx_query_set_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def pattern_batch_arrays(snapshot, q_type, inc_off, inc, has_ordered, pat_off, pat) -> QueryResult:
    """Packed batch (hgx_pattern_batch_packed): query q = And(type(q_type[q]),
    incident(inc[inc_off[q]:inc_off[q+1]]...), orderedLink(pat[pat_off[q]:pat_off[q+1]]) if has_ordered[q])."""
    n = len(q_type)
    arrs = [np.ascontiguousarray(q_type, np.int32), np.ascontiguousarray(inc_off, np.int64),
            np.ascontiguousarray(inc, np.int32), np.ascontiguousarray(has_ordered, np.int32),
            np.ascontiguousarray(pat_off, np.int64), np.ascontiguousarray(pat, np.int32)]
    h = C.c_void_p()
    check(lib().hgx_pattern_batch_packed(snapshot.handle, n, *(a.ctypes.data for a in arrs), C.byref(h)))
    return _read_result(h, n)


def pattern_batch_ext_arrays(snapshot, type_off, types, inc_off, inc, pos_off, pos, pset_off, pat_off, pat,
                             arity) -> QueryResult:
    """Flat batch for hgx_pattern_batch_ext (see include/hgx.h)."""
    n = len(arity)
    arrs = [np.ascontiguousarray(type_off, np.int64), np.ascontiguousarray(types, np.int32),
            np.ascontiguousarray(inc_off, np.int64), np.ascontiguousarray(inc, np.int32),
            np.ascontiguousarray(pos_off, np.int64), np.ascontiguousarray(pos, np.int32),
            np.ascontiguousarray(pset_off, np.int64), np.ascontiguousarray(pat_off, np.int64),
            np.ascontiguousarray(pat, np.int32), np.ascontiguousarray(arity, np.int32)]
    h = C.c_void_p()
    check(lib().hgx_pattern_batch_ext(snapshot.handle, n, *(a.ctypes.data for a in arrs), C.byref(h)))
    try:
        off = np.zeros(n + 1, np.int64)
        check(lib().hgx_query_result_offsets(h, ptr(off)))
        ids = np.zeros(max(int(off[-1]), 1), np.int32)
        check(lib().hgx_query_result_ids(h, ptr(ids)))
        a, b, c = C.c_double(), C.c_double(), C.c_double()
        check(lib().hgx_query_result_ms(h, C.byref(a), C.byref(b), C.byref(c)))
    finally:
        lib().hgx_query_result_free(h)
    return QueryResult(off, ids[: int(off[-1])], {"ms_total": a.value, "ms_match": b.value, "bytes_match": c.value})


def pattern_batch(snapshot, queries) -> QueryResult:
    """Evaluate many accelerated And queries in one GPU launch sequence.  ``queries``: conditions,
    normalised dicts, or legacy (type, incident, pattern) tuples (pattern None = no orderedLink)."""
    norm = []
    for q in queries:
        if isinstance(q, tuple):
            q = _from_tuple(q)
        elif not isinstance(q, dict) and q != "empty":
            q = normalize(q)
        norm.append(q)
    n = len(norm)
    type_off, inc_off, pos_off, pset_off = (np.zeros(n + 1, np.int64) for _ in range(4))
    types, inc, pos, pat, pat_off = [], [], [], [], [0]
    arity = np.full(n, -1, np.int32)
    empty = np.zeros(n, bool)
    for i, q in enumerate(norm):
        if q == "empty":   # nothing can match: run a NOP (an empty orderedLink) on a valid anchor
            empty[i] = True
            q = {"types": [], "inc": [0], "pos": [], "patterns": [()], "arity": -1}
        types.extend(q["types"])
        type_off[i + 1] = len(types)
        inc.extend(q["inc"])
        inc_off[i + 1] = len(inc)
        for rec in q["pos"]:
            pos.extend(rec)
        pos_off[i + 1] = len(pos) // 4
        for p in q["patterns"]:
            pat.extend(p)
            pat_off.append(len(pat))
        pset_off[i + 1] = len(pat_off) - 1
        arity[i] = q["arity"]
    r = pattern_batch_ext_arrays(snapshot, type_off, np.array(types or [0], np.int32), inc_off,
                                 np.array(inc or [0], np.int32), pos_off, np.array(pos or [0], np.int32), pset_off,
                                 np.array(pat_off, np.int64), np.array(pat or [0], np.int32), arity)
    if empty.any():
        parts = [np.empty(0, np.int32) if empty[i] else r[i] for i in range(n)]
        off = np.concatenate([[0], np.cumsum([len(p) for p in parts])]).astype(np.int64)
        return QueryResult(off, np.concatenate(parts).astype(np.int32), r.ms)
    return r


class QueryMetaData:
    """C/query/cond2qry/QueryMetaData.java -- ORACCESS for the accelerated And."""

    def __init__(self, ordered=True, random_access=True, predicate_cost=-1):
        self.ordered, self.randomAccess, self.predicateCost = ordered, random_access, predicate_cost


class GpuAndToQuery:
    """ConditionToQuery for And, registered with HGQueryConfiguration.addCompiler(And, ...)."""

    def getQuery(self, snapshot, cond):
        norm = normalize(cond)

        class _Q:
            def execute(_self):
                return list(pattern_batch(snapshot, [norm])[0].tolist())

        return _Q()

    def getMetaData(self, snapshot, cond):
        normalize(cond)
        return QueryMetaData(True, True, -1)


class HGQueryConfiguration:
    """Per-graph compiler registry (C/query/HGQueryConfiguration.java:37-66)."""

    def __init__(self):
        self._compilers = {}

    def addCompiler(self, cls, compiler):
        self._compilers[cls] = compiler

    def compiler(self, cls):
        return self._compilers.get(cls)


def find_all(snapshot, cond, config: HGQueryConfiguration | None = None):
    """hg.findAll(graph, cond) for the accelerated shapes."""
    if isinstance(cond, BFSCondition):
        # TraversalBasedQuery(traversal, ReturnType.targets) (ToQueryMap.java:313-319): the atoms
        # in HGBreadthFirstTraversal.next() order
        gen = DefaultALGenerator(snapshot, cond.link_predicate, None, *cond.flags)
        seq = bfs_sequence(snapshot, [cond.start], cond.max_distance, gen)
        return seq.pairs(0)[1].tolist()
    if isinstance(cond, MapCondition):
        return sorted({v for v in (cond.mapping(x) for x in find_all(snapshot, cond.cond, config)) if v is not None})
    if isinstance(cond, And):
        subs = _flatten(cond, [])
        if any(isinstance(c, (MapCondition, BFSCondition)) for c in subs):
            # And of mapped / traversal sub-queries: set intersection of the parts
            sets = [set(find_all(snapshot, c, config)) for c in subs if isinstance(c, (MapCondition, BFSCondition))]
            rest = [c for c in subs if not isinstance(c, (MapCondition, BFSCondition))]
            if rest:
                sets.append(set(find_all(snapshot, And(rest), config)))
            return sorted(set.intersection(*sets))
    compiler = (config.compiler(And) if config else None) or GpuAndToQuery()
    return compiler.getQuery(snapshot, cond).execute()
