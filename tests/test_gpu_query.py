"""GPU parity: batched And{type, incident, orderedLink} queries through the C ABI against the
oracle (literal ZigZagIntersectionResult restatement) -- identical ascending result sets."""
import json
import os

import numpy as np
import pytest

import kat_graphs as K
from oracle_ctypes import OracleGraph

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def snapshot(g):
    from hypergraphdb_amd import HyperGraphSnapshot
    return HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g.get("link_type"))


def oracle(g):
    return OracleGraph(g["num_atoms"], np.asarray(g["link_atom"], np.int32), np.asarray(g["tgt_off"], np.int64),
                       np.asarray(g["tgt_idx"], np.int32), np.asarray(g["link_type"], np.int32))


def test_kat_ordered_link_and_incident():
    """TC/query/Queries.java:131-140, 178-206."""
    from hypergraphdb_amd import find_all, hg, pattern_batch
    g = K.queries_graph()
    snap = snapshot(g)
    n = g["names"]
    assert find_all(snap, hg.and_(hg.type(K.T_TESTLINK), hg.orderedLink(n["n0"], n["n1"]))) == [n["linkH"]]
    assert find_all(snap, hg.incident(n["linkH"])) == [n["linkH1"]]
    assert find_all(snap, hg.incident(n["empty"])) == []
    # the truth table through the engine: and(incident(n0), orderedLink(p)) restricted to linkH
    res = pattern_batch(snap, [(K.T_TESTLINK, [n["n0"], n["n1"]], tuple(p)) for p, _ in K.ordered_link_truth_table(g)])
    for q, (p, expected) in enumerate(K.ordered_link_truth_table(g)):
        got = n["linkH"] in res[q].tolist()
        assert got == (expected and len(p) > 0), p   # an empty orderedLink compiles to HGQuery.NOP in an And


def test_kat_common_adjacency_pattern():
    """TC/query/PatternTests.java:20-61: {C1, C4} (hg.type(String) is implied: every atom is a string)."""
    from hypergraphdb_amd import find_all, hg
    g = K.pattern_graph()
    snap = snapshot(g)
    n = g["names"]
    cond = hg.and_(hg.apply(hg.targetAt(snap, 0), hg.orderedLink(hg.anyHandle(), n["A"])),
                   hg.apply(hg.targetAt(snap, 0), hg.orderedLink(hg.anyHandle(), n["B"])))
    L = find_all(snap, cond)
    assert n["C1"] in L and n["C4"] in L
    assert n["C2"] not in L and n["C3"] not in L and n["C5"] not in L


def test_kat_variable_incident_sets():
    """TC/query/QueryCompilation.java:35-73."""
    from hypergraphdb_amd import find_all, hg
    g = K.compilation_graph()
    snap = snapshot(g)
    n = g["names"]
    assert {n["l1"], n["l3"]} <= set(find_all(snap, hg.incident(n["h1"])))
    assert {n["l2"], n["l3"]} <= set(find_all(snap, hg.incident(n["h2"])))


def test_random_fixture_queries():
    from hypergraphdb_amd import pattern_batch
    d = np.load(os.path.join(GOLD, "random_small.npz"))
    gi = 0
    while f"g{gi}_A" in d:
        g = dict(num_atoms=int(d[f"g{gi}_A"][0]), link_atom=d[f"g{gi}_link_atom"], tgt_off=d[f"g{gi}_tgt_off"],
                 tgt_idx=d[f"g{gi}_tgt_idx"], link_type=d[f"g{gi}_link_type"])
        snap = snapshot(g)
        keys = json.loads(str(d[f"g{gi}_q_keys"]))
        qs, exp = [], []
        pos, res_all = 0, d[f"g{gi}_q_res"].tolist()
        for k in keys:
            t, ni, m, nr = k[:4]
            qs.append((t, k[4:4 + ni], None if m < 0 else tuple(k[4 + ni:4 + ni + m])))
            exp.append(res_all[pos:pos + nr])
            pos += nr
        if qs:
            r = pattern_batch(snap, qs)
            for q in range(len(qs)):
                assert r[q].tolist() == exp[q], (gi, qs[q])
        gi += 1


@pytest.mark.parametrize("case", range(4))
def test_random_queries_vs_oracle(case):
    from hypergraphdb_amd import pattern_batch
    rng = np.random.default_rng(900 + case)
    g = K.random_graph(rng, 400, 4000, max_arity=8, n_types=3, link_targets=case % 2 == 0)
    snap, orc = snapshot(g), oracle(g)
    qs = []
    for _ in range(3000):
        t = int(rng.integers(-1, 3))
        inc = [int(x) for x in rng.integers(0, g["num_atoms"], int(rng.integers(0, 4)))]
        m = int(rng.integers(-1, 5))
        pat = None if m < 0 else tuple(int(x) if rng.random() < 0.7 else -1 for x in rng.integers(0, 400, m))
        if not inc and not (pat and any(p >= 0 for p in pat)):
            inc = [int(rng.integers(0, g["num_atoms"]))]
        qs.append((t, inc, pat))
    r = pattern_batch(snap, qs)
    for q, (t, inc, pat) in enumerate(qs):
        assert r[q].tolist() == orc.and_query(t, inc, pat).tolist(), qs[q]


def test_config3_scaled_vs_oracle():
    """Config 3 shape at 0.5% scale: 3000 generated queries (degree-biased anchors, 10% negatives)."""
    from hypergraphdb_amd import pattern_batch, synth
    g = synth.config3(scale=0.005, n_queries=3000)
    snap, orc = snapshot(g), oracle(g)
    Q = g["queries"]
    qs = [(int(Q["type"][i]), [int(Q["a"][i])], (int(Q["x"][i]), -1, int(Q["y"][i]))) for i in range(3000)]
    r = pattern_batch(snap, qs)
    hits = 0
    for q, (t, inc, pat) in enumerate(qs):
        exp = orc.and_query(t, inc, pat)
        assert r[q].tolist() == exp.tolist(), q
        hits += len(exp) > 0
    assert hits > 2000          # most queries are positives (the sampled link matches)


def test_unsupported_and_empty_shapes():
    from hypergraphdb_amd import HGXUnsupported, pattern_batch
    g = K.queries_graph()
    snap = snapshot(g)
    with pytest.raises(HGXUnsupported):
        pattern_batch(snap, [(K.T_TESTLINK, [], None)])          # type scan: stays on AndToQuery
    with pytest.raises(HGXUnsupported):
        pattern_batch(snap, [(-1, [], (-1, -1))])
    r = pattern_batch(snap, [(-1, [g["names"]["n0"]], ())])      # empty orderedLink -> NOP
    assert r[0].tolist() == []


# --- extended And: PositionedIncident / Link / Arity / TypePlus / several orderedLinks ---------

def test_positioned_kat_through_engine():
    """TC/query/Queries.java:208-221 testPositionedLinkCondition (and hg.incidentNotAt)."""
    from hypergraphdb_amd import find_all, hg
    g = K.positioned_graph()
    snap = snapshot(g)
    links = {g["names"][f"L{i}"] for i in range(5)}
    for x, lb, ub, comp, contains, empty in K.positioned_truth_table(g):
        cond = hg.incidentNotAt(x, lb, ub) if comp else hg.incidentAt(x, lb, ub)
        got = find_all(snap, cond)
        assert (links <= set(got)) if contains else not (links & set(got)), (x, lb, ub, comp)
        if empty:
            assert got == []


def test_link_arity_and_multiple_patterns():
    from hypergraphdb_amd import find_all, hg
    g = K.queries_graph()
    snap, orc = snapshot(g), oracle(g)
    n = g["names"]
    assert find_all(snap, hg.and_(hg.link(n["n0"], n["n1"]), hg.arity(2))) == [n["linkH"]]
    assert find_all(snap, hg.and_(hg.link(n["n0"], n["n1"]), hg.arity(3))) == []
    assert find_all(snap, hg.and_(hg.incident(n["n2"]), hg.arity(3))) == [n["linkH1"]]
    assert find_all(snap, hg.and_(hg.arity(2), hg.arity(3), hg.incident(n["n0"]))) == []
    q = hg.and_(hg.orderedLink(n["n4"], hg.anyHandle(), n["n6"]), hg.orderedLink(n["n2"], n["linkH1"]))
    assert find_all(snap, q) == [n["link5"]]
    assert find_all(snap, q) == orc.and_query_ext([], [], [], [(n["n4"], -1, n["n6"]), (n["n2"], n["linkH1"])]).tolist()


@pytest.mark.parametrize("case", range(4))
def test_ext_random_vs_oracle(case):
    """Random extended Ands (type sets, incident, positioned, 0-2 orderedLinks, arity) on graphs with
    links targeting links and repeated targets: identical ascending result sets."""
    from hypergraphdb_amd import pattern_batch
    rng = np.random.default_rng(1200 + case)
    g = K.random_graph(rng, 300, 3000, max_arity=8, n_types=5, link_targets=case % 2 == 0)
    snap, orc = snapshot(g), oracle(g)
    A = g["num_atoms"]
    qs, exp = [], []
    while len(qs) < 2000:
        types = sorted({int(t) for t in rng.integers(0, 5, int(rng.integers(0, 3)))})
        inc = [int(x) for x in rng.integers(0, A, int(rng.integers(0, 3)))]
        pos = [(int(rng.integers(0, A)), int(rng.integers(-5, 6)), int(rng.integers(-5, 6)), int(rng.integers(0, 2)))
               for _ in range(int(rng.integers(0, 3)))]
        pats = [tuple(int(x) if rng.random() < 0.6 else -1 for x in rng.integers(0, A, int(rng.integers(1, 4))))
                for _ in range(int(rng.integers(0, 3)))]
        ar = int(rng.integers(-1, 7))
        e = orc.and_query_ext(types, inc, pos, pats, ar)
        if e is None:
            continue   # no incidence anchor: stays on AndToQuery (HGX_E_UNSUPPORTED)
        qs.append({"types": types, "inc": inc, "pos": pos, "patterns": pats, "arity": ar})
        exp.append(e.tolist())
    r = pattern_batch(snap, qs)
    for q in range(len(qs)):
        assert r[q].tolist() == exp[q], qs[q]


def test_type_plus_from_subsumption():
    """hg.and(hg.typePlus(base), hg.incident(a)): the subtypes come from a GPU HGSubsumes closure
    (TypePlusCondition.fetchSubTypes, C/query/TypePlusCondition.java:26-43)."""
    from hypergraphdb_amd import find_all, hg
    from hypergraphdb_amd.query import TypePlusCondition
    from oracle_ctypes import algen
    b = K.Builder()
    S = 9                                             # HGSubsumes type key
    tys = [b.node(f"T{i}") for i in range(6)]         # type atoms; key of T_i is i
    for gen_, spec in ((0, 1), (0, 2), (1, 3), (3, 4)):
        b.link(None, S, tys[gen_], tys[spec])         # HGSubsumes(general, specific)
    x = [b.node(f"x{i}") for i in range(8)]
    rng = np.random.default_rng(4)
    for i in range(60):
        t = int(rng.integers(0, 6))
        b.link(None, t, *[int(v) for v in rng.choice(x, int(rng.integers(1, 5)), replace=False)])
    g = b.arrays()
    snap, orc = snapshot(g), oracle(g)
    key_of = {tys[i]: i for i in range(6)}
    tp = TypePlusCondition.from_subsumption(snap, tys[1], S, key_of)
    assert tp.types == {1, 3, 4}
    lv = orc.bfs_levels(tys[0], -1, algen(S, False, True, False, False))
    assert TypePlusCondition.from_subsumption(snap, tys[0], S, key_of).types == {key_of[int(a)] for l in lv for a in l}
    for a in x:
        got = find_all(snap, hg.and_(hg.typePlus(tp), hg.incident(a)))
        assert got == orc.and_query_ext(sorted(tp.types), [a]).tolist()
        both = find_all(snap, hg.and_(hg.typePlus(tp), hg.type(3), hg.incident(a)))
        assert both == orc.and_query_ext([3], [a]).tolist()
        assert find_all(snap, hg.and_(hg.typePlus(tp), hg.type(2), hg.incident(a))) == []


def _packed(qs):
    """(type, [incident], pattern|None) list -> hgx_pattern_batch_packed arrays."""
    t = np.array([q[0] for q in qs], np.int32)
    inc_off = np.zeros(len(qs) + 1, np.int64)
    pat_off = np.zeros(len(qs) + 1, np.int64)
    inc, pat, ho = [], [], np.zeros(len(qs), np.int32)
    for i, (_, a, p) in enumerate(qs):
        inc += list(a)
        inc_off[i + 1] = len(inc)
        if p is not None:
            ho[i] = 1
            pat += list(p)
        pat_off[i + 1] = len(pat)
    return t, inc_off, np.array(inc, np.int32), ho, pat_off, np.array(pat, np.int32)


def test_packed_large_batch_vs_oracle():
    """A packed batch above the single-workgroup scan size (device scans + chunk map path),
    normalised on the device, against the oracle."""
    from hypergraphdb_amd import synth
    from hypergraphdb_amd.query import pattern_batch_arrays
    g = synth.config3(scale=0.01, n_queries=20000)
    snap, orc = snapshot(g), oracle(g)
    Q = g["queries"]
    rng = np.random.default_rng(31)
    qs = []
    for i in range(20000):
        if i % 4 == 3:   # untyped, two anchors, no pattern; or a repeated anchor (toDNF dedupe)
            a = int(Q["a"][i])
            qs.append((-1, [a, int(Q["x"][i]), a], None))
        else:
            qs.append((int(Q["type"][i]), [int(Q["a"][i])], (int(Q["x"][i]), -1, int(Q["y"][i]))))
    r = pattern_batch_arrays(snap, *_packed(qs))
    for q in rng.choice(len(qs), 3000, replace=False):
        t, inc, pat = qs[q]
        assert r[q].tolist() == orc.and_query(t, inc, pat).tolist(), qs[q]


def test_packed_workspace_growth():
    """Queries whose candidate ranges exceed the initial workspace are re-run with a grown one; the
    next batch reuses it.  Anchored on the highest-degree atoms, untyped."""
    from hypergraphdb_amd import synth
    from hypergraphdb_amd.query import pattern_batch_arrays
    g = synth.config3(scale=0.01, n_queries=10)
    snap, orc = snapshot(g), oracle(g)
    deg = np.diff(np.searchsorted(np.sort(g["tgt_idx"]), np.arange(g["num_atoms"] + 1)))
    hubs = np.argsort(-deg)[:3]
    assert deg[hubs[0]] > 16 * 3 + 4096
    for rep in range(2):
        qs = [(-1, [int(h)], None) for h in hubs]
        r = pattern_batch_arrays(snap, *_packed(qs))
        for q, (t, inc, pat) in enumerate(qs):
            assert r[q].tolist() == orc.and_query(t, inc, pat).tolist()


def test_packed_errors():
    from hypergraphdb_amd import HGXError, HGXUnsupported, _lib
    from hypergraphdb_amd.query import pattern_batch_arrays
    g = K.queries_graph()
    snap = snapshot(g)
    n0 = g["names"]["n0"]
    with pytest.raises(HGXError) as e:          # atom id out of range
        pattern_batch_arrays(snap, *_packed([(-1, [n0], None), (-1, [g["num_atoms"] + 5], None)]))
    assert e.value.code == _lib.HGX_E_INVALID and "query 1" in str(e.value)
    with pytest.raises(HGXUnsupported):         # no incidence anchor
        pattern_batch_arrays(snap, *_packed([(-1, [n0], None), (K.T_TESTLINK, [], (-1, -1))]))
    r = pattern_batch_arrays(snap, *_packed([(-1, [n0], ()), (-1, [n0], None)]))   # empty orderedLink: NOP
    assert r[0].tolist() == [] and len(r[1]) > 0


def _same(r1, r2, n):
    assert np.array_equal(r1.offsets, r2.offsets)
    for q in range(n):
        assert r1[q].tolist() == r2[q].tolist(), q


def test_packed_batches_vs_oracle_and_removed_fused_path():
    """Packed batches against the oracle: typed orderedLink queries, untyped multi-anchor queries with
    repeated anchors, hub anchors with thousands of hits (result-area growth), empty orderedLinks
    (NOP), several batches in a row, and a batch with a 70-entry anchor list.  The fused small-batch
    path (HGX_OPT_QUERY_FUSED 1, measured slower) was removed in round 5: only 0 is accepted."""
    from hypergraphdb_amd import HGXError, _lib, synth
    from hypergraphdb_amd.query import pattern_batch_arrays
    g = synth.config3(scale=0.01, n_queries=6000)
    snap, orc = snapshot(g), oracle(g)
    Q = g["queries"]
    deg = np.diff(np.searchsorted(np.sort(g["tgt_idx"]), np.arange(g["num_atoms"] + 1)))
    hubs = [int(h) for h in np.argsort(-deg)[:4]]
    rng = np.random.default_rng(77)
    qs = []
    for i in range(6000):
        k = i % 10
        if k < 6:
            qs.append((int(Q["type"][i]), [int(Q["a"][i])], (int(Q["x"][i]), -1, int(Q["y"][i]))))
        elif k < 8:
            a = int(Q["a"][i])
            qs.append((-1, [a, int(Q["x"][i]), a], None))
        elif k == 8:
            qs.append((int(Q["type"][i]), [hubs[i % 4]], None) if i % 20 == 8 else (-1, [int(Q["a"][i])], ()))
        else:
            qs.append((-1, [hubs[(i // 10) % 4]], (int(Q["x"][i]),)))
    arrs = _packed(qs)
    first = pattern_batch_arrays(snap, *arrs)
    again = pattern_batch_arrays(snap, *arrs)
    _same(first, again, len(qs))
    assert max(len(first[q]) for q in range(len(qs))) > 64
    for q in rng.choice(len(qs), 600, replace=False):
        t, inc, pat = qs[q]
        assert first[q].tolist() == orc.and_query(t, inc, pat).tolist(), qs[q]
    long_q = (-1, [int(Q["a"][0])] * 70, None)
    r1 = pattern_batch_arrays(snap, *_packed(qs[:100] + [long_q]))
    for q in range(100):
        assert r1[q].tolist() == first[q].tolist(), q
    assert r1[100].tolist() == orc.and_query(-1, [int(Q["a"][0])], None).tolist()
    snap.set_option(_lib.HGX_OPT_QUERY_FUSED, 0)
    with pytest.raises(HGXError) as ei:
        snap.set_option(_lib.HGX_OPT_QUERY_FUSED, 1)
    assert ei.value.code == _lib.HGX_E_UNSUPPORTED


@pytest.mark.parametrize("case", range(2))
def test_inline_records_vs_tgt_rows_and_oracle(case):
    """HGX_OPT_QUERY_INLINE: typed candidates read their link's targets from the 32-byte inline record
    of the type-grouped index (links of arity > 8 fall back to tgt_off).  Single-type extended Ands
    (positioned, several orderedLinks, arity) on links of arity 0-12: inline on, inline off and the
    oracle give identical ascending result sets."""
    from hypergraphdb_amd import _lib, pattern_batch
    rng = np.random.default_rng(1500 + case)
    g = K.random_graph(rng, 300, 3000, max_arity=12, n_types=4, link_targets=case == 0)
    snap, orc = snapshot(g), oracle(g)
    A = g["num_atoms"]
    qs, exp = [], []
    while len(qs) < 2000:
        types = [int(rng.integers(0, 4))]
        inc = [int(x) for x in rng.integers(0, A, int(rng.integers(1, 3)))]
        pos = [(int(rng.integers(0, A)), int(rng.integers(-9, 10)), int(rng.integers(-9, 10)), int(rng.integers(0, 2)))
               for _ in range(int(rng.integers(0, 2)))]
        pats = [tuple(int(x) if rng.random() < 0.6 else -1 for x in rng.integers(0, A, int(rng.integers(1, 5))))
                for _ in range(int(rng.integers(0, 3)))]
        ar = int(rng.integers(-1, 13))
        e = orc.and_query_ext(types, inc, pos, pats, ar)
        if e is None:
            continue
        qs.append({"types": types, "inc": inc, "pos": pos, "patterns": pats, "arity": ar})
        exp.append(e.tolist())
    # plain typed queries too (the packed entry point, registers-only pattern path)
    plain = [(int(rng.integers(0, 4)), [int(rng.integers(0, A))],
              tuple(int(x) if rng.random() < 0.7 else -1 for x in rng.integers(0, A, int(rng.integers(1, 6)))))
             for _ in range(2000)]
    plain_exp = [orc.and_query(t, i, p).tolist() for t, i, p in plain]
    for inline in (1, 0, 1):
        snap.set_option(_lib.HGX_OPT_QUERY_INLINE, inline)
        r = pattern_batch(snap, qs)
        for q in range(len(qs)):
            assert r[q].tolist() == exp[q], (inline, qs[q])
        r = pattern_batch(snap, plain)
        for q in range(len(plain)):
            assert r[q].tolist() == plain_exp[q], (inline, plain[q])


def test_single_pass_match_vs_oracle():
    """The single-pass pipeline (front-scan and match kernels with decoupled look-backs) gives the
    oracle's results: batches with long runs of queries without candidates (a chunk window of more
    than 64 queries), empty orderedLinks, untyped and typed queries, and a batch above 16384 queries.
    HGX_OPT_QUERY_FLAT 0 / 1 (the per-query chunks and the separate-scan flat back end, measured
    slower) were removed in round 5 and are refused."""
    from hypergraphdb_amd import HGXError, _lib, pattern_batch
    rng = np.random.default_rng(1700)
    g = K.random_graph(rng, 400, 4000, max_arity=8, n_types=3, link_targets=True)
    snap, orc = snapshot(g), oracle(g)
    A = g["num_atoms"]
    isolated = [a for a in range(A) if orc.and_query(-1, [a], None).size == 0][:5]
    assert isolated
    qs = []
    for i in range(20000):
        r = rng.random()
        if r < 0.3:   # no candidates: an anchor without incidence, or an empty orderedLink
            qs.append((-1, [isolated[i % len(isolated)]], None) if i % 3 else (-1, [int(rng.integers(0, A))], ()))
        else:
            t = int(rng.integers(-1, 3))
            pat = None if rng.random() < 0.5 else tuple(int(x) if rng.random() < 0.7 else -1
                                                        for x in rng.integers(0, A, int(rng.integers(1, 4))))
            qs.append((t, [int(rng.integers(0, A))], pat))
    for lo, hi in ((0, 3000), (3000, 3300), (0, 20000)):
        sub = qs[lo:hi]
        exp = [orc.and_query(t, i, p).tolist() for t, i, p in sub]
        r = pattern_batch(snap, sub)
        for q in range(len(sub)):
            assert r[q].tolist() == exp[q], (lo + q, sub[q])
    for flat in (0, 1):
        with pytest.raises(HGXError) as ei:
            snap.set_option(_lib.HGX_OPT_QUERY_FLAT, flat)
        assert ei.value.code == _lib.HGX_E_UNSUPPORTED
    snap.set_option(_lib.HGX_OPT_QUERY_FLAT, 2)


def test_single_pass_packed_batches_all_sizes():
    """The single-pass pipeline on the packed entry (device normalisation in the front-scan kernel):
    batch sizes 1..70000 (1 to 274 front blocks; chunk counts from 0 to thousands, so both look-backs
    run across many predecessors), batches whose queries all have no candidate, the workspace-growth
    re-run, and the same results when the batch runs again."""
    from hypergraphdb_amd import _lib
    from hypergraphdb_amd.query import pattern_batch_arrays
    rng = np.random.default_rng(1900)
    g = K.random_graph(rng, 3000, 30000, max_arity=8, n_types=4, link_targets=True)
    snap, orc = snapshot(g), oracle(g)
    A = g["num_atoms"]
    off, tg, lt = g["tgt_off"], g["tgt_idx"], g["link_type"]

    def batch(n):
        ty, inc, pat, po, ho = [], [], [], [0], []
        for _ in range(n):
            r = int(rng.integers(0, len(off) - 1))
            t = tg[off[r]:off[r + 1]]
            a = int(t[int(rng.integers(0, len(t)))]) if len(t) and rng.random() < 0.8 else int(rng.integers(0, A))
            ty.append(int(lt[r]) if rng.random() < 0.6 else -1)
            inc.append(a)
            if len(t) >= 3 and rng.random() < 0.5:
                pat += [int(t[0]), -1, int(t[2])]
                ho.append(1)
            else:
                ho.append(0)
            po.append(len(pat))
        return (np.array(ty, np.int32), np.arange(n + 1, dtype=np.int64), np.array(inc, np.int32),
                np.array(ho, np.int32), np.array(po, np.int64), np.array(pat, np.int32))

    for n in (1, 2, 63, 255, 256, 257, 1000, 5000, 70000):
        b = batch(n)
        ref = None
        for rep in range(2):
            r = pattern_batch_arrays(snap, *b)
            if ref is None:
                ref = r
                if n <= 5000:
                    for q in range(n):
                        p = b[5][b[4][q]:b[4][q + 1]].tolist() if b[3][q] else None
                        e = orc.and_query(int(b[0][q]), [int(b[2][q])], p)
                        assert r.ids[r.offsets[q]:r.offsets[q + 1]].tolist() == e.tolist(), (n, q)
            else:
                assert np.array_equal(r.offsets, ref.offsets) and np.array_equal(r.ids, ref.ids), n
    # every query without candidates (isolated anchors): zero chunks, all offsets 0
    isolated = np.array([a for a in range(A) if orc.and_query(-1, [a], None).size == 0][:50], np.int32)
    n = len(isolated)
    r = pattern_batch_arrays(snap, np.full(n, -1, np.int32), np.arange(n + 1, dtype=np.int64), isolated,
                             np.zeros(n, np.int32), np.zeros(n + 1, np.int64), np.zeros(0, np.int32))
    assert r.offsets.tolist() == [0] * (n + 1)


def test_query_set_resident_batches():
    """hgx_query_set_create + hgx_pattern_batch_set: a packed batch uploaded once and run repeatedly,
    in every front-end mode, on the snapshot and on an execution context of it, equals the packed
    call (and the oracle), also into caller buffers (hgx_pattern_batch_set_into); bad offsets are
    refused at creation."""
    from hypergraphdb_amd import HGXError, _lib
    from hypergraphdb_amd.query import QuerySet, pattern_batch_arrays
    from hypergraphdb_amd import synth
    g = synth.config3(scale=0.002, n_queries=3000)
    snap, orc = snapshot(g), oracle(g)
    Q = g["queries"]
    nq = len(Q["type"])
    packed = (Q["type"], np.arange(nq + 1, dtype=np.int64), Q["a"], np.ones(nq, np.int32),
              np.arange(0, 3 * nq + 1, 3, dtype=np.int64),
              np.stack([Q["x"], np.full(nq, -1, np.int32), Q["y"]], 1).reshape(-1))
    ref = pattern_batch_arrays(snap, *packed)
    for q in range(0, nq, 101):
        assert ref[q].tolist() == orc.and_query(int(Q["type"][q]), [int(Q["a"][q])],
                                                (int(Q["x"][q]), -1, int(Q["y"][q]))).tolist()
    qs = QuerySet(snap, *packed)
    ctx = snap.context()
    for flat in (2,):
        for target in (snap, ctx):
            for _ in range(2):
                r = qs.run(target)
                assert np.array_equal(r.offsets, ref.offsets) and np.array_equal(r.ids, ref.ids), (flat, target is ctx)
            # caller buffers (hgx_pattern_batch_set_into): exact fit, then too small (offsets and the
            # count still come back, the ids array is left alone)
            total = int(ref.offsets[-1])
            off = np.full(nq + 1, -7, np.int64)
            ids = np.full(total + 3, -7, np.int32)
            tm = np.full(3, -1.0)
            assert qs.run_into(target, off, ids, tm) == total
            assert np.array_equal(off, ref.offsets) and np.array_equal(ids[:total], ref.ids)
            assert (tm >= 0).all()
            assert (ids[total:] == -7).all()
            off[:] = -7
            small = np.full(max(total - 1, 0), -7, np.int32)
            assert qs.run_into(target, off, small) == total
            assert np.array_equal(off, ref.offsets) and (small == -7).all()
    with pytest.raises(ValueError):
        qs.run_into(snap, np.zeros(nq, np.int64), np.zeros(8, np.int32))
    qs.close()
    bad = list(packed)
    bad[1] = np.arange(1, nq + 2, dtype=np.int64)   # inc_off[0] != 0
    with pytest.raises(HGXError):
        QuerySet(snap, *bad)
    ctx.close()
    snap.close()


def test_placement_query_ranges_at_block_starts():
    """The placement kernel writes the result offsets of the queries starting in its 64 chunks (4096
    candidates): its query range starts one past the owner of the candidate before the block, or --
    when a query's candidates begin exactly at the block start -- at the first of the candidate-free
    queries before it (a ballot over 64 queries at a time).  Untyped one-anchor queries have exactly
    deg(anchor) candidates, so the batch is built to put a query start exactly on block starts, after
    runs of 1, 63, 64, 65, 130 and 300 candidate-free queries, with such runs at the batch's head and
    tail too; single-pass results equal the oracle's and the flat path's offsets."""
    from hypergraphdb_amd import _lib
    from hypergraphdb_amd.query import pattern_batch_arrays
    N, S = 2000, 50                      # node atoms (deg(v) = v % 98), sink atoms
    link_atom, tgt_off, tgt_idx = [], [0], []
    for v in range(N):
        for j in range(v % 98):
            link_atom.append(N + S + len(link_atom))
            tgt_idx += [v, N + (v * 7 + j) % S]
            tgt_off.append(len(tgt_idx))
    M = len(link_atom)
    g = {"num_atoms": N + S + M, "link_atom": np.array(link_atom, np.int32), "tgt_off": np.array(tgt_off, np.int64),
         "tgt_idx": np.array(tgt_idx, np.int32), "link_type": np.ones(M, np.int32)}
    snap, orc = snapshot(g), oracle(g)
    by_deg = {}
    for v in range(N):
        by_deg.setdefault(v % 98, []).append(v)
    iso = by_deg[0]
    anchors, total, block = [], 0, 64 * 64
    anchors += [iso[i % len(iso)] for i in range(150)]
    rng = np.random.default_rng(2024)
    for run in (1, 63, 64, 65, 130, 300, 7):
        target = (total // block + 2) * block   # fill to a block start exactly, then the run
        while total < target:
            d = min(97, target - total, int(rng.integers(20, 98)))
            anchors.append(by_deg[d][int(rng.integers(0, len(by_deg[d])))])
            total += d
        anchors += [iso[i % len(iso)] for i in range(run)]
    for _ in range(40):
        d = int(rng.integers(1, 98))
        anchors.append(by_deg[d][0])
    anchors += [iso[i % len(iso)] for i in range(150)]
    n = len(anchors)
    b = (np.full(n, -1, np.int32), np.arange(n + 1, dtype=np.int64), np.array(anchors, np.int32),
         np.zeros(n, np.int32), np.zeros(n + 1, np.int64), np.zeros(0, np.int32))
    r2 = pattern_batch_arrays(snap, *b)
    cache = {}
    for q, a in enumerate(anchors):
        if a not in cache:
            cache[a] = orc.and_query(-1, [a], None).tolist()
        assert r2.ids[r2.offsets[q]:r2.offsets[q + 1]].tolist() == cache[a], (q, a)
    assert r2.offsets[-1] == sum(a % 98 for a in anchors)
    # every query's hits are its candidates here, so the offsets show the alignment the batch was built for:
    # a query with candidates starting exactly on a block start right after a candidate-free run
    aligned = [q for q in range(1, n) if anchors[q] % 98 and anchors[q - 1] % 98 == 0 and r2.offsets[q] > 0
               and r2.offsets[q] % block == 0]
    assert len(aligned) >= 6, aligned


def test_large_candidate_batch_placement_prefix():
    """A batch whose candidate space spans more than 256 placement blocks (> 16384 chunks of 64
    candidates) takes the scanned block prefix in the placement (hgx_q_place_bsum / _bscan) instead of
    every block summing all chunks before it (quadratic); results equal the oracle's for a
    sample and a second run's."""
    import time
    from hypergraphdb_amd import _lib
    from hypergraphdb_amd.query import pattern_batch_arrays
    from hypergraphdb_amd import synth
    g = synth.hypergraph(2000, 400000, 2, 5, 1.6, 2, seed=11)
    snap, orc = snapshot(g), oracle(g)
    deg = np.bincount(g["tgt_idx"], minlength=g["num_atoms"])
    hubs = np.argsort(-deg)[:64].astype(np.int32)
    rng = np.random.default_rng(5)
    nq = 6000
    anchors = hubs[rng.integers(0, len(hubs), nq)]
    types = np.where(rng.random(nq) < 0.5, -1, rng.integers(0, 2, nq)).astype(np.int32)
    args = (types, np.arange(nq + 1, dtype=np.int64), anchors, np.zeros(nq, np.int32),
            np.zeros(nq + 1, np.int64), np.zeros(0, np.int32))
    assert int(sum(deg[anchors])) > 64 * 64 * 260   # > 260 placement blocks of candidates
    b = pattern_batch_arrays(snap, *args)
    t0 = time.perf_counter()
    a = pattern_batch_arrays(snap, *args)
    print(f"large batch: single-pass {(time.perf_counter() - t0) * 1e3:.3f} ms")
    assert np.array_equal(a.offsets, b.offsets) and np.array_equal(a.ids, b.ids)
    for q in range(0, nq, 97):
        assert a[q].tolist() == orc.and_query(int(types[q]), [int(anchors[q])], None).tolist(), q
