"""CPU tests: the oracle against the reference's known-answer tests and the golden fixtures, and
the two independent restatements (C oracle, Python pyref) against each other."""
import itertools
import json
import os

import numpy as np
import pytest

import kat_graphs as K
import pyref
from oracle_ctypes import OracleGraph, algen, ordered_link

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def og(g):
    return OracleGraph(g["num_atoms"], np.asarray(g["link_atom"], np.int32), np.asarray(g["tgt_off"], np.int64),
                       np.asarray(g["tgt_idx"], np.int32), np.asarray(g["link_type"], np.int32))


def pg(g):
    links = {}
    off, tg = np.asarray(g["tgt_off"]), np.asarray(g["tgt_idx"])
    for r, la in enumerate(np.asarray(g["link_atom"]).tolist()):
        links[la] = (int(np.asarray(g["link_type"])[r]), tg[off[r]:off[r + 1]].tolist())
    return pyref.Graph(list(range(g["num_atoms"])), links)


def bfs_seq(o, seed, maxd, mode, lt=-1):
    P, S, R, RS = mode
    l, a, d, _ = o.bfs(seed, -1 if maxd is None else maxd, algen(lt, P, S, R, RS))
    return list(zip(l.tolist(), a.tolist(), d.tolist()))


# ---------------------------------------------------------------- reference KATs
def test_kat_linkage_bfs_reaches_x3():
    """TC/links/TestLinkage.java:58-66: hg.and(hg.bfs(x1), hg.is(x3)) finds x3."""
    g = K.linkage_graph()
    n = g["names"]
    seq = bfs_seq(og(g), n["x1"], None, K.ALGEN_MODES[0])
    assert n["x3"] in [a for _, a, _ in seq]
    assert (n["l2"], n["x3"], 2) in seq


def test_kat_incident_condition():
    """TC/query/Queries.java:131-140: incident(empty link) has no result; incident(linkH) count == 1."""
    g = K.queries_graph()
    n, o = g["names"], og(g)
    assert o.incidence(n["empty"]).tolist() == []
    assert o.incidence(n["linkH"]).tolist() == [n["linkH1"]]
    assert o.and_query(-1, [n["linkH"]]).tolist() == [n["linkH1"]]


def test_kat_ordered_link_condition():
    """TC/query/Queries.java:178-206: findAll(and(linkType, orderedLink(n0, n1))) == [linkH] + truth table."""
    g = K.queries_graph()
    n, o = g["names"], og(g)
    assert o.and_query(K.T_TESTLINK, [], [n["n0"], n["n1"]]).tolist() == [n["linkH"]]
    targets = [n["n0"], n["n1"]]
    for pattern, expected in K.ordered_link_truth_table(g):
        assert ordered_link(targets, pattern) == expected, pattern
        assert pyref.ordered_link(targets, pattern) == expected


def test_kat_bfs_condition_counts():
    """TC/query/Queries.java:336-361: BFS from linkH returns as many links as targets (one pair each)."""
    g = K.queries_graph()
    n, o = g["names"], og(g)
    seq = bfs_seq(o, n["linkH"], None, K.ALGEN_MODES[0])
    links = [l for l, _, _ in seq]
    targets = [a for _, a, _ in seq]
    assert len(links) == len(targets) == len(set(targets)) > 0
    # linkH is reachable only through linkH1 (its sole incident link)
    assert seq[0][0] == n["linkH1"]


def test_kat_pattern_common_adjacency():
    """TC/query/PatternTests.java:20-61: apply(targetAt(0), orderedLink(ANY, A)) and the same for B
    intersect to {C1, C4}."""
    g = K.pattern_graph()
    n, o = g["names"], og(g)
    tg = lambda l: np.asarray(g["tgt_idx"])[np.asarray(g["tgt_off"])[l - n["p0"]]]  # noqa: E731  (link rows p0..)
    to_a = {int(tg(l)) for l in o.and_query(-1, [], [-1, n["A"]]).tolist()}
    to_b = {int(tg(l)) for l in o.and_query(-1, [], [-1, n["B"]]).tolist()}
    both = to_a & to_b
    assert n["C1"] in both and n["C4"] in both
    assert n["C2"] not in both and n["C3"] not in both and n["C5"] not in both


def test_kat_variable_incident_sets():
    """TC/query/QueryCompilation.java:35-73: incident(h1) contains l1, l3; incident(h2) contains l2, l3."""
    g = K.compilation_graph()
    n, o = g["names"], og(g)
    assert {n["l1"], n["l3"]} <= set(o.incidence(n["h1"]).tolist())
    assert {n["l2"], n["l3"]} <= set(o.incidence(n["h2"]).tolist())


# ---------------------------------------------------------------- golden fixtures
def test_oracle_matches_kat_fixture():
    with open(os.path.join(GOLD, "kat.json")) as f:
        kat = json.load(f)
    for name, e in kat.items():
        o = og(e)
        for a, inc in e["incidence"].items():
            assert o.incidence(int(a)).tolist() == inc
        for key, seq in e["bfs"].items():
            a, mi, maxd = key.split("/")
            got = bfs_seq(o, int(a), None if maxd == "None" else int(maxd), K.ALGEN_MODES[int(mi)])
            assert got == [tuple(x) for x in seq], (name, key)


def test_oracle_matches_random_fixture():
    d = np.load(os.path.join(GOLD, "random_small.npz"))
    gi = 0
    while f"g{gi}_A" in d:
        g = dict(num_atoms=int(d[f"g{gi}_A"][0]), link_atom=d[f"g{gi}_link_atom"], tgt_off=d[f"g{gi}_tgt_off"],
                 tgt_idx=d[f"g{gi}_tgt_idx"], link_type=d[f"g{gi}_link_type"])
        o = og(g)
        pos = 0
        seq_all = d[f"g{gi}_bfs_seq"]
        for seed, mi, lt, maxd, n in d[f"g{gi}_bfs_keys"].tolist():
            got = bfs_seq(o, seed, None if maxd < 0 else maxd, K.ALGEN_MODES[mi], lt)
            assert got == [tuple(x) for x in seq_all[pos:pos + n].tolist()]
            pos += n
        qpos = 0
        res = d[f"g{gi}_q_res"]
        for k in json.loads(str(d[f"g{gi}_q_keys"])):
            t, ni, m, nr = k[:4]
            inc = k[4:4 + ni]
            pat = None if m < 0 else k[4 + ni:4 + ni + m]
            assert o.and_query(t, inc, pat).tolist() == res[qpos:qpos + nr].tolist()
            qpos += nr
        gi += 1
    assert gi >= 10


def test_config1_fixture_reproduces():
    """The config-1 graph regenerated by the product generator is the one the fixture pins
    (SHA-256), and the oracle reproduces the per-depth sets of all 64 seeds."""
    import hashlib

    from hypergraphdb_amd import synth
    d = np.load(os.path.join(GOLD, "config1.npz"))
    g = synth.config1()
    h = hashlib.sha256()
    for k in ("link_atom", "tgt_off", "tgt_idx"):
        h.update(np.ascontiguousarray(g[k]).tobytes())
    assert h.hexdigest() == str(d["graph_sha256"])
    assert np.array_equal(g["seeds"], d["seeds"])
    o = OracleGraph(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    off, ids = d["level_off"], d["level_ids"]
    k = 0
    for s in g["seeds"].tolist():
        lv = o.bfs_levels(s, 3)
        for depth in range(4):
            exp = ids[off[k]:off[k + 1]]
            got = lv[depth] if depth < len(lv) else np.empty(0, np.int32)
            assert np.array_equal(got, exp)
            k += 1


# ---------------------------------------------------------------- restatements agree
@pytest.mark.parametrize("gi", range(6))
def test_c_oracle_equals_pyref_random(gi):
    rng = np.random.default_rng(1000 + gi)
    g = K.random_graph(rng, int(rng.integers(5, 60)), int(rng.integers(3, 60)), link_targets=gi % 2 == 0)
    o, p = og(g), pg(g)
    for a in range(g["num_atoms"]):
        for mode in K.ALGEN_MODES:
            lt = int(rng.integers(-1, 3))
            P, S, R, RS = mode
            assert [tuple(x) for x in pyref.generate(p, a, link_type=None if lt < 0 else lt, preceding=P,
                                                     succeeding=S, reverse=R, source=RS)] == \
                o.generate(a, algen(lt, *mode))
            maxd = [None, 1, 2, 4][a % 4]
            assert bfs_seq(o, a, maxd, mode, lt) == pyref.bfs(p, a, maxd, link_type=None if lt < 0 else lt,
                                                              preceding=P, succeeding=S, reverse=R, source=RS)


def test_zigzag_equals_set_intersection():
    """The literal ZigZagIntersectionResult restatement returns the sorted set intersection on every
    random query shape (so the GPU's set formulation is the reference's result)."""
    rng = np.random.default_rng(7)
    for _ in range(30):
        g = K.random_graph(rng, 30, 120, max_arity=6, n_types=2)
        o, p = og(g), pg(g)
        for _ in range(40):
            t = int(rng.integers(-1, 2))
            inc = [int(x) for x in rng.integers(0, g["num_atoms"], int(rng.integers(1, 4)))]
            m = int(rng.integers(-1, 4))
            pat = None if m < 0 else [int(x) if rng.random() < 0.6 else -1 for x in rng.integers(0, 30, m)]
            a = o.and_query(t, inc, pat)
            b = o.and_query(t, inc, pat, zigzag=False)
            c = pyref.and_query(p, None if t < 0 else t, inc, pat)
            assert a.tolist() == b.tolist() == list(c)


# ---------------------------------------------------------------- GPU neighbour rule
def test_closed_form_neighbour_rule_exhaustive():
    """pyref.reachable (the rule the HIP kernels implement) equals the DefaultALGenerator
    restatement on every target array of arity <= 5 over 4 symbols, every flag combination."""
    for arity in range(1, 6):
        for tg in itertools.product(range(4), repeat=arity):
            links = {10: (0, list(tg))}
            atoms = sorted(set(tg))
            g = pyref.Graph(atoms + [10], links)
            for mode in K.ALGEN_MODES:
                P, S, R, RS = mode
                m = pyref.mode_of(P, S, R, RS)
                for v in atoms:
                    got = {a for _, a in pyref.generate(g, v, preceding=P, succeeding=S, reverse=R, source=RS)}
                    got.discard(v)
                    want = {t for t in atoms if t != v and pyref.reachable(m, list(tg), v, t)}
                    assert got == want, (tg, mode, v)


# --- extended And: PositionedIncident / Link / Arity / TypePlus / several orderedLinks ---------

def _ext_graphs():
    g = K.positioned_graph()
    rg = [K.random_graph(np.random.default_rng(s), 120, 300, max_arity=7, n_types=4) for s in (5, 6)]
    return [g] + rg


def test_positioned_kat_queries_java():
    """TC/query/Queries.java:208-221 on both restatements."""
    import pyref
    g = K.positioned_graph()
    orc, pgr = og(g), pg(g)
    links = [g["names"][f"L{i}"] for i in range(5)]
    for x, lb, ub, comp, contains, empty in K.positioned_truth_table(g):
        got = orc.and_query_ext(positioned=[(x, lb, ub, int(comp))]).tolist()
        assert got == pyref.and_query_ext(pgr, positioned_=[(x, lb, ub, comp)])
        assert set(links) <= set(got) if contains else not (set(links) & set(got))
        if empty:
            assert got == []


def test_positioned_predicate_exhaustive():
    """og_positioned == pyref.positioned on every target array of arity <= 4 over 3 symbols."""
    import itertools
    import pyref
    from oracle_ctypes import positioned
    for n in range(0, 5):
        for row in itertools.product(range(3), repeat=n):
            for lb in range(-5, 5):
                for ub in range(-5, 5):
                    for c in (False, True):
                        assert positioned(row, 1, lb, ub, c) == pyref.positioned(list(row), 1, lb, ub, c)


def test_ext_queries_oracle_vs_pyref():
    import pyref
    for g in _ext_graphs():
        orc, pgr = og(g), pg(g)
        rng = np.random.default_rng(g["num_atoms"])
        A = g["num_atoms"]
        for _ in range(400):
            types = sorted({int(t) for t in rng.integers(0, 4, int(rng.integers(0, 3)))})
            inc = [int(x) for x in rng.integers(0, A, int(rng.integers(0, 3)))]
            pos = [(int(rng.integers(0, A)), int(rng.integers(-4, 5)), int(rng.integers(-4, 5)), int(rng.integers(0, 2)))
                   for _ in range(int(rng.integers(0, 3)))]
            pats = [tuple(int(x) if rng.random() < 0.6 else -1 for x in rng.integers(0, A, int(rng.integers(1, 4))))
                    for _ in range(int(rng.integers(0, 3)))]
            ar = int(rng.integers(-1, 6))
            a = orc.and_query_ext(types, inc, pos, pats, ar)
            b = pyref.and_query_ext(pgr, types, inc, pos, pats, ar if ar >= 0 else None)
            assert (a is None and b is None) or a.tolist() == b, (types, inc, pos, pats, ar)


def test_ext_reduces_to_base_and():
    """With one type and one pattern the extended And is the literal zig-zag And."""
    for g in _ext_graphs():
        orc = og(g)
        rng = np.random.default_rng(3)
        for _ in range(300):
            t = int(rng.integers(-1, 4))
            inc = [int(x) for x in rng.integers(0, g["num_atoms"], int(rng.integers(1, 3)))]
            pat = tuple(int(x) if rng.random() < 0.6 else -1 for x in rng.integers(0, g["num_atoms"], 3))
            a = orc.and_query_ext([] if t < 0 else [t], inc, [], [pat], -1)
            b = orc.and_query(t, inc, pat)
            assert a.tolist() == b.tolist()
