"""The reference's own known-answer test graphs, rebuilt as snapshots.

Handles follow IntHandleFactory (C/handle/IntHandleFactory.java:32,49): user atoms get
sequential handles in add order, so atom id = add order.  Type keys are arbitrary ints.
Paths: TC = testcore/test/java/hgtest in the reference.
"""
from __future__ import annotations

import numpy as np

T_NODE, T_VALUELINK, T_TESTLINK, T_PLAIN = 0, 1, 2, 3


class Builder:
    def __init__(self):
        self.n = 0
        self.names = {}
        self.links = []          # (atom, type, targets)

    def node(self, name):
        a = self.n
        self.n += 1
        self.names[name] = a
        return a

    def link(self, name, type_, *targets):
        a = self.n
        self.n += 1
        if name:
            self.names[name] = a
        self.links.append((a, type_, list(targets)))
        return a

    def arrays(self):
        link_atom = np.array([a for a, _, _ in self.links], np.int32)
        off = np.zeros(len(self.links) + 1, np.int64)
        tg = []
        for i, (_, _, t) in enumerate(self.links):
            tg += t
            off[i + 1] = len(tg)
        lt = np.array([t for _, t, _ in self.links], np.int32)
        return dict(num_atoms=self.n, link_atom=link_atom, tgt_off=off, tgt_idx=np.array(tg, np.int32),
                    link_type=lt, names=dict(self.names))


def linkage_graph():
    """TC/links/TestLinkage.java:58-66 testSimpleConnection: x1-x2-x3 via two plain links."""
    b = Builder()
    x1, x2, x3 = b.node("x1"), b.node("x2"), b.node("x3")
    b.link("l1", T_PLAIN, x1, x2)
    b.link("l2", T_PLAIN, x2, x3)
    return b.arrays()


def queries_graph():
    """TC/query/Queries.java:466-537 setUp: NestedBean n0..n9 (COUNT-1), one HGValueLink over all of
    them, the duplicated bean n10, then create_simple_subgraph: linkH=(n0,n1), linkH1=(n2,n3,linkH),
    an empty link, and (n4,n5,n6,n2,linkH1)."""
    b = Builder()
    nb = [b.node(f"n{i}") for i in range(10)]
    b.link("valuelink", T_VALUELINK, *nb)
    b.node("n10")
    linkH = b.link("linkH", T_TESTLINK, nb[0], nb[1])
    linkH1 = b.link("linkH1", T_TESTLINK, nb[2], nb[3], linkH)
    b.link("empty", T_TESTLINK)
    b.link("link5", T_TESTLINK, nb[4], nb[5], nb[6], nb[2], linkH1)
    return b.arrays()


def pattern_graph():
    """TC/query/PatternTests.java:20-61 testCommonAdjacencyPattern (the (c5,b) link is added twice)."""
    b = Builder()
    a, bb = b.node("A"), b.node("B")
    c = {k: b.node(k) for k in ("C1", "C2", "C3", "C4", "C5")}
    for i, (s, t) in enumerate([("C1", a), ("C1", bb), ("C1", c["C2"]), ("C2", a), ("C2", c["C3"]), ("C4", a),
                                ("C4", bb), ("C5", bb), ("C5", bb), ("C5", c["C2"])]):
        b.link(f"p{i}", T_PLAIN, c[s], t)
    return b.arrays()


def compilation_graph():
    """TC/query/QueryCompilation.java:35-73 testVariableReplacement: l1=(h1), l2=(h2), l3=(h1,h2)."""
    b = Builder()
    h1, h2 = b.node("h1"), b.node("h2")
    b.link("l1", T_PLAIN, h1)
    b.link("l2", T_PLAIN, h2)
    b.link("l3", T_PLAIN, h1, h2)
    return b.arrays()


def positioned_graph():
    """TC/query/Queries.java:208-221 testPositionedLinkCondition: ten atoms A0..A9 and five plain
    links over all of them in order (plus the queries graph's shape of an unrelated link)."""
    b = Builder()
    A = [b.node(f"A{i}") for i in range(10)]
    for i in range(5):
        b.link(f"L{i}", T_PLAIN, *A)
    b.link("other", T_TESTLINK, A[3], A[0])
    return b.arrays()


def positioned_truth_table(g):
    """(target, lower, upper, complement, contains all five links?, empty?) -- Queries.java:217-220,
    plus the complement forms of hg.incidentNotAt."""
    n = g["names"]
    return [(n["A0"], 0, 0, False, True, False), (n["A9"], -1, -1, False, True, False),
            (n["A5"], 3, 7, False, True, False), (n["A3"], -4, -1, False, False, True),
            (n["A3"], -4, -1, True, True, False), (n["A5"], 3, 7, True, False, True)]


def ordered_link_truth_table(g):
    """TC/query/Queries.java:178-206 on linkH = (n0, n1): (pattern, expected)."""
    n = g["names"]
    return [([], True), ([n["n5"]], False), ([n["n1"]], True), ([n["n0"], n["n1"]], True),
            ([n["n1"], n["n0"]], False)]


def random_graph(rng, n_nodes, n_links, max_arity=5, link_targets=True, repeat_p=0.15, n_types=3):
    """Small random hypergraphs exercising every edge case of the path: links targeting links,
    repeated targets inside a link, arity 0/1 links, empty incidence sets, several types.
    Atom ids are a random interleaving of nodes and links (rank order is arbitrary)."""
    A = n_nodes + n_links
    order = rng.permutation(A)
    is_link = np.zeros(A, bool)
    is_link[order[:n_links]] = True
    link_atoms = np.sort(order[:n_links]).astype(np.int32)
    off = [0]
    tg = []
    for la in link_atoms:
        k = int(rng.integers(0, max_arity + 1))
        row = []
        for _ in range(k):
            if row and rng.random() < repeat_p:
                row.append(row[int(rng.integers(0, len(row)))])
            else:
                cand = int(rng.integers(0, A))
                if not link_targets and is_link[cand]:
                    cand = int(rng.choice(np.nonzero(~is_link)[0]))
                if cand == la:          # a link cannot target itself
                    cand = (cand + 1) % A
                row.append(cand)
        tg += row
        off.append(len(tg))
    return dict(num_atoms=A, link_atom=link_atoms, tgt_off=np.array(off, np.int64),
                tgt_idx=np.array(tg, np.int32), link_type=rng.integers(0, n_types, n_links).astype(np.int32))


ALGEN_MODES = [
    # (preceding, succeeding, reverse, source)  -- 6-arg ctor forbids (False, False, *, no source)
    (True, True, False, False),
    (False, True, False, False),
    (True, False, False, False),
    (True, True, True, False),
    (False, True, True, False),
    (True, False, True, False),
    (True, True, False, True),
    (False, False, False, True),
    (True, False, False, True),
    (False, True, True, True),
    (True, False, True, True),
    (False, False, True, True),
]
