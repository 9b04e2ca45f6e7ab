"""TEST INFRASTRUCTURE, NOT PRODUCT CODE.

Second, independent restatement of the reference hot path in pure Python, used
only in this container to cross-check the C oracle (oracle/hgx_oracle.c) and to
generate the committed golden fixtures (tests/golden/make_golden.py).  Small
inputs only.  Paths are relative to the reference root;
C = core/src/java/org/hypergraphdb.

It is written against a different model than the C oracle: handles are kept
as opaque Python values in dicts (as the Java HashMap<HGHandle, ..> does), and
incidence sets are built from a per-atom Python set, then sorted.
"""
from __future__ import annotations

from collections import deque
from dataclasses import dataclass, field

ANY = -1  # hg.anyHandle() (IntHandleFactory.anyHandle, C/handle/IntHandleFactory.java:25,44)


@dataclass
class Graph:
    """Atoms are ints ordered like their persistent handles.  ``links`` maps a link
    atom to (type, targets) = its layout [type, value, t0..] without the value
    (C/HyperGraph.java:1603-1608)."""
    atoms: list
    links: dict = field(default_factory=dict)

    def __post_init__(self):
        inc = {a: set() for a in self.atoms}
        for l, (_, tg) in self.links.items():
            for t in tg:                          # putNoDupData: one entry per (t, l)
                inc[t].add(l)
        # sorted duplicates, unsigned byte order == handle order (BJE...:109-111)
        self.inc = {a: sorted(s) for a, s in inc.items()}

    def targets(self, l):
        return self.links[l][1]

    def type_of(self, l):
        return self.links[l][0]


class AdjIterator:
    """DefaultALGenerator.AdjIterator with siblingPredicate == null
    (C/algorithms/DefaultALGenerator.java:85-364)."""

    def __init__(self, g, src, link_type=None, preceding=True, succeeding=True,
                 reverse=False, source=False):
        self.g, self.src = g, src
        self.link_type = link_type
        self.P, self.S, self.R, self.RS = preceding, succeeding, reverse, source
        self.min_arity = 1 if source else 2
        self.it = iter(g.inc[src])
        self.cur = None
        self._next_link()

    # F/B TargetSetIterator ------------------------------------------------
    def _reset(self):
        t, src, n = self.tg, self.src, len(self.tg)
        self.seen = False
        if not self.R:
            self.pos = 0
            if not self.P:
                while True:
                    hit = t[self.pos] == src
                    self.pos += 1
                    if hit:
                        break
                self.seen = True
                if self.RS:
                    self.pos -= 1
                    return
                if self.pos == n:
                    self.pos = -1
                    return
            if not self.seen and t[self.pos] == src:
                self.seen = True
                if self.RS:
                    return
                if not self.S:
                    self.pos = -1
                    return
                self.pos += 1
        else:
            self.pos = n - 1
            if not self.P:
                while True:
                    hit = t[self.pos] == src
                    self.pos -= 1
                    if hit:
                        break
                self.seen = True
                if self.RS:
                    self.pos += 1
                    return
                if self.pos == -1:
                    return
            if not self.seen and t[self.pos] == src:
                self.seen = True
                if self.RS:
                    return
                if not self.S:
                    self.pos = -1
                    return
                self.pos -= 1

    def _advance(self):
        t, src, n = self.tg, self.src, len(self.tg)
        if not self.R:
            self.pos += 1
            if self.pos == n:
                self.pos = -1
                return
            if not self.seen and t[self.pos] == src:
                self.seen = True
                if self.RS:
                    return
                if not self.S:
                    self.pos = -1
                    return
                self.pos += 1
                if self.pos == n:
                    self.pos = -1
        else:
            self.pos -= 1
            if self.pos == -1:
                return
            if not self.seen and t[self.pos] == src:
                self.seen = True
                if self.RS:
                    return
                if not self.S:
                    self.pos = -1
                else:
                    self.pos -= 1

    def _next_link(self):
        for l in self.it:
            if self.link_type is not None and self.g.type_of(l) != self.link_type:
                continue
            self.tg = self.g.targets(l)
            if len(self.tg) < self.min_arity:
                continue
            self._reset()
            if self.pos != -1:
                self.cur = l
                return
        self.cur = None

    def __iter__(self):
        while self.cur is not None:
            l = self.cur
            a = self.tg[self.pos]
            self._advance()
            if self.pos == -1:
                self._next_link()
            yield l, a


def generate(g, src, **opts):
    return list(AdjIterator(g, src, **opts))


def bfs(g, seed, max_dist=None, **opts):
    """HGBreadthFirstTraversal drained through next() (C/algorithms/HGBreadthFirstTraversal.java).
    Returns [(link, atom, dist)] in FIFO order."""
    maxd = float("inf") if max_dist is None or max_dist < 0 else max_dist
    examined = {seed: True}
    q = deque()
    out = []

    def advance(frm, d):
        if d >= maxd:
            return
        for l, a in AdjIterator(g, frm, **opts):
            if a not in examined:
                q.append((l, a, d + 1))
                examined[a] = False

    advance(seed, 0)
    while q:
        l, a, d = q.popleft()
        examined[a] = True
        out.append((l, a, d))
        advance(a, d)
    return out


def per_depth_sets(seq, seed, levels):
    sets = [set() for _ in range(levels)]
    sets[0].add(seed)
    for _, a, d in seq:
        if d < levels:
            sets[d].add(a)
    return [sorted(s) for s in sets]


def ordered_link(targets, pattern):
    """OrderedLinkCondition.satisfies (C/query/OrderedLinkCondition.java:92-124)."""
    i = j = 0
    while i < len(targets) and j < len(pattern):
        if pattern[j] == ANY or pattern[j] == targets[i]:
            j += 1
        i += 1
    return j == len(pattern)


def and_query(g, type_=None, incident=(), pattern=None):
    """Set semantics of And(type, incident.., orderedLink) after
    ExpressionBasedQuery.expand (:730-737).  None = not accelerated (no anchor)."""
    anchors = []
    for h in list(incident) + [p for p in (pattern or []) if p != ANY]:
        if h not in anchors:
            anchors.append(h)
    if not anchors:
        return None
    if pattern is not None and len(pattern) == 0:
        return []          # QueryMetaData.EMPTY goes into ORA; its query is HGQuery.NOP
    cand = set(g.inc[anchors[0]])
    for a in anchors[1:]:
        cand &= set(g.inc[a])
    res = []
    for l in sorted(cand):
        if type_ is not None and g.type_of(l) != type_:
            continue
        if pattern is not None and not ordered_link(g.targets(l), pattern):
            continue
        res.append(l)
    return res


def positioned(targets, x, lb, ub, complement=False):
    """PositionedIncidentCondition.satisfies (C/query/PositionedIncidentCondition.java:123-177)."""
    n = len(targets)
    if ub < 0:
        ub += n
    if lb < 0:
        lb += n
    if lb > ub or lb < 0 or ub < 0 or lb >= n or ub >= n:
        return False
    inside = [i for i in range(n) if targets[i] == x and lb <= i <= ub]
    outside = [i for i in range(n) if targets[i] == x and not lb <= i <= ub]
    return bool(outside) if complement else bool(inside)


def and_query_ext(g, types=(), incident=(), positioned_=(), patterns=(), arity=None):
    """Set semantics of the extended And: Or over types (TypePlusCondition), incident anchors (also
    LinkCondition / orderedLink targets), position-filtered incidence sets, every orderedLink and
    the arity as predicates.  None = not accelerated (no anchor)."""
    anchors = []
    for h in list(incident) + [p for pat in patterns for p in pat if p != ANY]:
        if h not in anchors:
            anchors.append(h)
    if not anchors and not positioned_:
        return None
    if any(len(p) == 0 for p in patterns):
        return []
    sets = [set(g.inc[a]) for a in anchors]
    for (x, lb, ub, c) in positioned_:
        sets.append({l for l in g.inc[x] if positioned(g.targets(l), x, lb, ub, c)})
    cand = set.intersection(*sets)
    res = []
    for l in sorted(cand):
        if types and g.type_of(l) not in set(types):
            continue
        if arity is not None and arity >= 0 and len(g.targets(l)) != arity:
            continue
        if not all(ordered_link(g.targets(l), p) for p in patterns):
            continue
        res.append(l)
    return res


# ----------------------------------------------------------------------------
# Closed-form neighbour rule used by the GPU kernels.
# Tested exhaustively against AdjIterator above (tests/test_oracle.py).
# ----------------------------------------------------------------------------

MODE_SYM, MODE_AFTER_FIRST, MODE_BEFORE_FIRST, MODE_BEFORE_LAST, MODE_AFTER_LAST = range(5)


def mode_of(preceding=True, succeeding=True, reverse=False, source=False):
    if not reverse:
        if not preceding:
            return MODE_AFTER_FIRST
        if not succeeding and not source:
            return MODE_BEFORE_FIRST
        return MODE_SYM
    if not preceding:
        return MODE_BEFORE_LAST
    if not succeeding and not source:
        return MODE_AFTER_LAST
    return MODE_SYM


def reachable(mode, targets, v, t):
    """True iff atom t (!= v) is yielded by generate(v) through a link with these
    targets (both v and t occur in it)."""
    fv = targets.index(v)
    lv = len(targets) - 1 - targets[::-1].index(v)
    ft = targets.index(t)
    lt = len(targets) - 1 - targets[::-1].index(t)
    if mode == MODE_SYM:
        return True
    if mode == MODE_AFTER_FIRST:
        return lt > fv
    if mode == MODE_BEFORE_FIRST:
        return ft < fv
    if mode == MODE_BEFORE_LAST:
        return ft < lv
    return lt > lv
