"""GPU parity: batched BFS through the C ABI against the oracle / golden fixtures (bit-exact
per-depth visited sets)."""
import json
import os

import numpy as np
import pytest

import kat_graphs as K
from oracle_ctypes import OracleGraph, algen

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def snapshot(g):
    from hypergraphdb_amd import HyperGraphSnapshot
    return HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g.get("link_type"))


def oracle(g):
    return OracleGraph(g["num_atoms"], np.asarray(g["link_atom"], np.int32), np.asarray(g["tgt_off"], np.int64),
                       np.asarray(g["tgt_idx"], np.int32),
                       None if g.get("link_type") is None else np.asarray(g["link_type"], np.int32))


def gen(snap, mode, lt=-1):
    from hypergraphdb_amd import AtomTypeCondition, DefaultALGenerator
    P, S, R, RS = mode
    return DefaultALGenerator(snap, None if lt < 0 else AtomTypeCondition(lt), None, P, S, R, RS)


def levels_from_seq(seed, seq):
    d = {0: [seed]}
    for _, a, k in seq:
        d.setdefault(k, []).append(a)
    n = max(d) + 1
    return [sorted(d.get(k, [])) for k in range(n)]


def gpu_levels(res, i):
    lv = [res.visited(i, d).tolist() for d in range(res.n_levels)]
    while len(lv) > 1 and not lv[-1]:
        lv.pop()
    return lv


def check_batch(g, seeds, maxd, mode, lt=-1, snap=None, orc=None):
    from hypergraphdb_amd import bfs_batch
    snap = snap or snapshot(g)
    orc = orc or oracle(g)
    res = bfs_batch(snap, seeds, maxd, gen(snap, mode, lt))
    counts = res.counts()
    for i, s in enumerate(seeds):
        l, a, d, _ = orc.bfs(int(s), -1 if maxd is None else maxd, algen(lt, *mode))
        exp = levels_from_seq(int(s), zip(l.tolist(), a.tolist(), d.tolist()))
        got = gpu_levels(res, i)
        assert got == exp, (i, s, mode, maxd, lt)
        assert counts[i, :len(exp)].tolist() == [len(x) for x in exp]
        assert counts[i, len(exp):].sum() == 0
    res.close()


def test_kat_fixture_graphs_every_seed_every_mode():
    with open(os.path.join(GOLD, "kat.json")) as f:
        kat = json.load(f)
    for name, e in kat.items():
        g = {k: np.asarray(v) if isinstance(v, list) else v for k, v in e.items() if k not in ("bfs", "incidence")}
        snap = snapshot(g)
        from hypergraphdb_amd import bfs_batch
        seeds = list(range(g["num_atoms"]))
        for a, inc in e["incidence"].items():
            assert snap.incidence(int(a)).tolist() == inc
        for mi, mode in enumerate(K.ALGEN_MODES):
            for maxd in (None, 1, 2):
                res = bfs_batch(snap, seeds, maxd, gen(snap, mode))
                for s in seeds:
                    exp = levels_from_seq(s, e["bfs"][f"{s}/{mi}/{maxd}"])
                    assert gpu_levels(res, s) == exp, (name, s, mode, maxd)
                res.close()
        snap.close()


def test_kat_linkage_reaches_x3():
    from hypergraphdb_amd import find_all, hg
    g = K.linkage_graph()
    snap = snapshot(g)
    assert g["names"]["x3"] in find_all(snap, hg.bfs(g["names"]["x1"]))


def test_random_fixture_graphs():
    d = np.load(os.path.join(GOLD, "random_small.npz"))
    gi = 0
    while f"g{gi}_A" in d:
        g = dict(num_atoms=int(d[f"g{gi}_A"][0]), link_atom=d[f"g{gi}_link_atom"], tgt_off=d[f"g{gi}_tgt_off"],
                 tgt_idx=d[f"g{gi}_tgt_idx"], link_type=d[f"g{gi}_link_type"])
        snap = snapshot(g)
        from hypergraphdb_amd import bfs_batch
        pos = 0
        seq_all = d[f"g{gi}_bfs_seq"].tolist()
        for seed, mi, lt, maxd, n in d[f"g{gi}_bfs_keys"].tolist():
            res = bfs_batch(snap, [seed], None if maxd < 0 else maxd, gen(snap, K.ALGEN_MODES[mi], lt))
            assert gpu_levels(res, 0) == levels_from_seq(seed, seq_all[pos:pos + n])
            pos += n
            res.close()
        snap.close()
        gi += 1


def test_config1_golden_all_64_seeds():
    """64 seeds, depth 3, per-depth sets bit-identical to the fixture."""
    from hypergraphdb_amd import bfs_batch, synth
    fx = np.load(os.path.join(GOLD, "config1.npz"))
    g = synth.config1()
    snap = snapshot(g)
    res = bfs_batch(snap, g["seeds"], 3)
    off, ids = fx["level_off"], fx["level_ids"]
    k = 0
    for i in range(64):
        for depth in range(4):
            exp = ids[off[k]:off[k + 1]]
            got = res.visited(i, depth) if depth < res.n_levels else np.empty(0, np.int32)
            assert np.array_equal(got, exp), (i, depth)
            k += 1


@pytest.mark.parametrize("case", range(8))
def test_random_graphs_all_modes_multi_batch(case):
    """Links targeting links, repeated targets, arity 0/1 links, random rank interleaving, typed link
    predicates, duplicate seeds, batches not a multiple of 64 and > 1024 seeds (several batches)."""
    rng = np.random.default_rng(500 + case)
    g = K.random_graph(rng, int(rng.integers(200, 2000)), int(rng.integers(200, 3000)), max_arity=7,
                       link_targets=case % 2 == 0, n_types=3)
    snap, orc = snapshot(g), oracle(g)
    mode = K.ALGEN_MODES[case % len(K.ALGEN_MODES)]
    n_seeds = [1, 63, 64, 65, 200, 1024, 1100, 2100][case]
    seeds = rng.integers(0, g["num_atoms"], n_seeds).astype(np.int32)
    lt = [-1, 0, 1, -1, 2, -1, 0, -1][case]
    maxd = [None, 2, 3, None, 1, 4, None, 2][case]
    check_batch(g, seeds, maxd, mode, lt, snap, orc)


def test_heavy_atoms_power_law():
    """Hubs with > 512 incident links take the chunked workgroup path; results stay exact."""
    from hypergraphdb_amd import synth
    g = synth.hypergraph(3000, 20000, 2, 8, 2.1, 3, seed=11)
    deg = np.bincount(g["tgt_idx"], minlength=g["num_atoms"])
    assert deg.max() > 4096            # several chunks for the top hub
    snap, orc = snapshot(g), oracle(g)
    seeds = np.concatenate([np.arange(5), np.arange(2900, 3000)]).astype(np.int32)
    for mode in (K.ALGEN_MODES[0], K.ALGEN_MODES[1], K.ALGEN_MODES[4]):
        check_batch(g, seeds, 3, mode, -1, snap, orc)
    check_batch(g, seeds, None, K.ALGEN_MODES[0], 1, snap, orc)


def test_config2_scaled_counts_and_sets():
    """Config 2 shape (Chung-Lu gamma 2.1, arity 2..8) at 1% scale, 1024 seeds, depth 4:
    every seed's per-depth counts equal the oracle's; full sets for 6 sampled seeds."""
    from hypergraphdb_amd import bfs_batch, synth
    g = synth.config2(scale=0.01)
    snap, orc = snapshot(g), oracle(g)
    res = bfs_batch(snap, g["seeds"], 4)
    counts = res.counts()
    oc, trav = orc.bfs_many(g["seeds"], 4, 5)
    assert np.array_equal(counts[:, :5], oc)
    st = res.stats()
    assert st["traversed_edges"] == float(trav.sum())      # the TEPS numerator is exact
    for i in (0, 1, 100, 511, 512, 1023):
        lv = orc.bfs_levels(int(g["seeds"][i]), 4)
        for d_, exp in enumerate(lv):
            assert np.array_equal(res.visited(i, d_), exp), (i, d_)


def test_subsumption_config5_scaled():
    """hg.subsumed / hg.subsumes: unbounded BFS over HGSubsumes links only (ToQueryMap.java:282-370)."""
    from hypergraphdb_amd import AtomTypeCondition, DefaultALGenerator, bfs_batch, synth
    g = synth.config5(scale=0.002, n_sources=300)
    snap, orc = snapshot(g), oracle(g)
    T = g["subsumes_type"]
    for reverse in (False, True):
        gen_ = DefaultALGenerator(snap, AtomTypeCondition(T), None, False, True, reverse)
        res = bfs_batch(snap, g["seeds"], None, gen_)
        counts = res.counts()
        oc, _ = orc.bfs_many(g["seeds"], -1, res.n_levels + 1, algen(T, False, True, reverse, False))
        assert np.array_equal(counts, oc[:, :res.n_levels])
        assert oc[:, res.n_levels:].sum() == 0
        for i in (0, 7, 299):
            lv = orc.bfs_levels(int(g["seeds"][i]), -1, algen(T, False, True, reverse, False))
            for d_, exp in enumerate(lv):
                assert np.array_equal(res.visited(i, d_), exp)
        res.close()


def test_traversal_api_and_is_visited():
    from hypergraphdb_amd import DefaultALGenerator, HGBreadthFirstTraversal
    g = K.queries_graph()
    snap = snapshot(g)
    n = g["names"]
    tr = HGBreadthFirstTraversal(n["linkH"], DefaultALGenerator(snap))
    seen = []
    while tr.hasNext():
        link, atom = tr.next()
        assert atom in snap.targets(link).tolist()
        assert tr.isVisited(atom)
        seen.append(atom)
    orc = oracle(g)
    _, a, _, _ = orc.bfs(n["linkH"], -1)
    assert sorted(seen) == sorted(a.tolist())
    with pytest.raises(NotImplementedError):
        tr.remove()


def test_depth_of_and_errors():
    from hypergraphdb_amd import HGXError, bfs_batch
    g = K.queries_graph()
    snap = snapshot(g)
    res = bfs_batch(snap, [g["names"]["n0"], g["names"]["n10"]], None)
    assert res.depth_of(0, g["names"]["n0"]) == 0
    assert res.depth_of(0, g["names"]["n1"]) == 1
    assert res.depth_of(1, g["names"]["n0"]) == -1      # n10 has no incident link
    assert res.counts()[1].tolist()[:1] == [1]
    with pytest.raises(HGXError):
        bfs_batch(snap, [g["num_atoms"]], 2)
    with pytest.raises(HGXError):
        res.visited(5, 0)


@pytest.mark.parametrize("flags", [0x0, 0x1, 0x2, 0x4, 0x8, 0xF, 0xE, 0x28, 0x3E, 0x7E, 0x40, 0xBE, 0x13E, 0x1BE, 0x1B6, 0x3BE, 0x236, 0xBBE,
                                   0x13BE, 0x23BE, 0x43BE, 0x73BE, 0x83BE, 0x83BA, 0xF3BA, 0x0BBE,
                                   0x203BE, 0x2003E, 0x20008, 0x2000A, 0x203BA, 0x223BE])
def test_engine_option_matrix(flags):
    """Every work-avoidance option (early exits, full-visited skipping, frontier-driven sparse
    levels) returns the same per-depth sets; power-law hubs + random edge cases + ordered modes."""
    from hypergraphdb_amd import _lib, synth
    cases = []
    rng = np.random.default_rng(77)
    cases.append((K.random_graph(rng, 800, 2500, max_arity=7, n_types=3), K.ALGEN_MODES[0], -1, None))
    cases.append((K.random_graph(rng, 800, 2500, max_arity=7, n_types=3), K.ALGEN_MODES[4], 1, 3))
    cases.append((synth.hypergraph(3000, 20000, 2, 8, 2.1, 3, seed=12), K.ALGEN_MODES[0], -1, 3))
    cases.append((synth.hypergraph(3000, 20000, 2, 8, 2.1, 3, seed=13), K.ALGEN_MODES[1], 2, None))
    for i, (g, mode, lt, maxd) in enumerate(cases):
        snap, orc = snapshot(g), oracle(g)
        snap.set_option(_lib.HGX_OPT_BFS_FLAGS, flags)
        snap.set_option(_lib.HGX_OPT_BFS_BLOCK, 0)   # the rows engine's variants (not the workgroup stage)
        seeds = rng.integers(0, g["num_atoms"], 1024 if i == 2 else 300).astype(np.int32)   # W = 16 and W < 16
        check_batch(g, seeds, maxd, mode, lt, snap, orc)


def test_engine_flags_reject_internal_bits():
    """Bits 16+ are the engine's per-level internal flags (kAllRows): hgx_set_option refuses them
    (-1 as 'everything on' used to switch the pull to the all-rows path)."""
    from hypergraphdb_amd import HGXError, _lib
    g = K.random_graph(np.random.default_rng(3), 50, 80)
    snap = snapshot(g)
    for bad in (-1, 1 << 16, 0x183BE, 1 << 18, 0x3FFFF):
        with pytest.raises(HGXError, match="bits 0-15"):
            snap.set_option(_lib.HGX_OPT_BFS_FLAGS, bad)
    snap.set_option(_lib.HGX_OPT_BFS_FLAGS, 0xFFFF)
    check_batch(g, np.arange(40, dtype=np.int32), None, K.ALGEN_MODES[0], -1, snap, oracle(g))
    snap.set_option(_lib.HGX_OPT_BFS_FLAGS, 0x2FFFF)   # bit 17 (frontier-code pull) is settable
    check_batch(g, np.arange(40, dtype=np.int32), None, K.ALGEN_MODES[0], -1, snap, oracle(g))


@pytest.mark.parametrize("n_seeds,lt", [(1024, -1), (300, -1), (1024, 1)])
def test_nonfull_pull_levels(n_seeds, lt):
    """Late dense levels where most incidence sits on atoms visited by every traversal run the
    non-full pull (level kind 3); per-depth sets stay identical to the oracle's, unbounded and
    with a link type."""
    from hypergraphdb_amd import _lib, bfs_batch, synth
    g = synth.hypergraph(3000, 20000, 2, 8, 2.1, 3, seed=14)
    snap, orc = snapshot(g), oracle(g)
    snap.set_option(_lib.HGX_OPT_BFS_BLOCK, 0)
    # seeds with (typed) incidence: every traversal covers the same component, so atoms become full
    off, tg = g["tgt_off"], g["tgt_idx"]
    rows = np.nonzero(g["link_type"] == lt)[0] if lt >= 0 else np.arange(len(off) - 1)
    has = np.zeros(g["num_atoms"], bool)
    for r in rows:
        has[tg[off[r]:off[r + 1]]] = True
    seeds = np.random.default_rng(15).choice(np.nonzero(has)[0], n_seeds, replace=False).astype(np.int32)
    res = bfs_batch(snap, seeds, None, gen(snap, K.ALGEN_MODES[0], lt))
    kinds = res.stats(accounting=False)["level_sparse"]
    res.close()
    assert 3 in kinds, kinds
    check_batch(g, seeds, None, K.ALGEN_MODES[0], lt, snap, orc)


@pytest.mark.parametrize("n_seeds,lt,scale", [(1024, -1, 8), (300, -1, 8), (1024, 1, 8), (1024, -1, 1), (512, 2, 1)])
def test_frontier_code_levels(n_seeds, lt, scale):
    """Dense levels over a small frontier run the frontier-code pull (level kind 4, HGX_OPT_BFS_FLAGS bit
    17): per-entry target records, frontier rows as <= 6-id codes or dense rows, hub chunks in registers.
    Per-depth sets equal the oracle's and the gather + pull engine's, with few-bit rows (a large graph
    per seed: codes) and many-bit rows (1024 seeds on a small graph: dense rows), typed and untyped."""
    from hypergraphdb_amd import _lib, bfs_batch, synth
    g = synth.hypergraph(3000 * scale, 20000 * scale, 2, 8, 2.1, 3, seed=21 + scale)
    snap, orc = snapshot(g), oracle(g)
    snap.set_option(_lib.HGX_OPT_BFS_BLOCK, 0)   # every seed on the rows engine
    seeds = np.random.default_rng(22).choice(3000 * scale, n_seeds, replace=False).astype(np.int32)
    sets = {}
    for flags in (0x203BE, 0x3BE):
        snap.set_option(_lib.HGX_OPT_BFS_FLAGS, flags)
        res = bfs_batch(snap, seeds, 4, gen(snap, K.ALGEN_MODES[0], lt))
        st = res.stats(accounting=False)
        assert (4 in st["level_sparse"]) == bool(flags & 0x20000), (flags, st["level_sparse"])
        if flags & 0x20000:
            assert st["kernels"]["hgx_fc_pull"]["launches"] >= 1
        sets[flags] = (res.counts(), [res.visited(i, d).tobytes() for i in range(0, n_seeds, 37) for d in range(5)])
        res.close()
    assert np.array_equal(sets[0x203BE][0], sets[0x3BE][0]) and sets[0x203BE][1] == sets[0x3BE][1]
    snap.set_option(_lib.HGX_OPT_BFS_FLAGS, 0x203BE)
    check_batch(g, seeds if n_seeds <= 512 else seeds[:: max(1, n_seeds // 96)], 4, K.ALGEN_MODES[0], lt, snap, orc)


def test_frontier_code_refused_for_long_links():
    """A snapshot with a link of arity > 8 has no frontier-code records: its dense levels keep gather + pull
    (no level of kind 4) and the sets stay exact."""
    from hypergraphdb_amd import _lib, bfs_batch
    rng = np.random.default_rng(23)
    g = K.random_graph(rng, 600, 3000, max_arity=12, n_types=1)
    snap, orc = snapshot(g), oracle(g)
    snap.set_option(_lib.HGX_OPT_BFS_BLOCK, 0)
    seeds = rng.integers(0, g["num_atoms"], 1024).astype(np.int32)
    res = bfs_batch(snap, seeds, 3, gen(snap, K.ALGEN_MODES[0]))
    assert 4 not in res.stats(accounting=False)["level_sparse"]
    res.close()
    check_batch(g, seeds[:200], 3, K.ALGEN_MODES[0], -1, snap, orc)


@pytest.mark.parametrize("batch", [0])
def test_push_batch_all_modes(batch):
    """The frontier push (one atom per wavefront) gives the oracle's per-depth sets in every generator
    mode: power-law hubs (heavy chunks), typed links, long rows (> 8 targets), links targeting links,
    300 and 1024 seeds.  HGX_OPT_PUSH_BATCH K > 0 (the flattened push, measured slower) was removed in
    round 5 and is refused."""
    from hypergraphdb_amd import HGXError, _lib, synth
    rng = np.random.default_rng(91)
    cases = [(K.random_graph(rng, 600, 2500, max_arity=12, n_types=3), -1, None, 300),
             (synth.hypergraph(3000, 20000, 2, 8, 2.1, 3, seed=17), 1, None, 1024),
             (synth.config5(scale=0.001, n_sources=300), None, None, 300)]
    for gi, (g, lt, maxd, ns) in enumerate(cases):
        snap, orc = snapshot(g), oracle(g)
        snap.set_option(_lib.HGX_OPT_PUSH_BATCH, batch)
        with pytest.raises(HGXError) as ei:
            snap.set_option(_lib.HGX_OPT_PUSH_BATCH, 8)
        assert ei.value.code == _lib.HGX_E_UNSUPPORTED
        snap.set_option(_lib.HGX_OPT_BFS_BLOCK, 0)
        if gi == 2:
            lt = int(g["subsumes_type"])
            modes = [(False, True, False, False), (False, True, True, False)]
            seeds = np.asarray(g["seeds"], np.int32)
        else:
            modes = K.ALGEN_MODES[::2] if gi == 0 else K.ALGEN_MODES[1::3]
            seeds = rng.integers(0, g["num_atoms"], ns).astype(np.int32)
        for mode in modes:
            check_batch(g, seeds, maxd, mode, lt, snap, orc)


def test_frontier_push_all_modes():
    """The frontier push (rows engine) gives the oracle's per-depth sets in every generator mode: rows
    longer than 8 targets (the loop past the register row), typed links, power-law hubs (chunked push),
    links targeting links, and the config-5 ontology in both subsumption directions.  HGX_OPT_PUSH_INLINE
    (inline target records, measured no faster, removed in round 5) accepts only 0."""
    from hypergraphdb_amd import HGXUnsupported, _lib, synth
    rng = np.random.default_rng(93)
    cases = [(K.random_graph(rng, 600, 2500, max_arity=12, n_types=3), -1, None, 300),
             (synth.hypergraph(3000, 20000, 2, 8, 2.1, 3, seed=19), 1, 3, 1024),
             (synth.config5(scale=0.002, n_sources=500), None, None, 500)]
    for gi, (g, lt, maxd, ns) in enumerate(cases):
        snap, orc = snapshot(g), oracle(g)
        snap.set_option(_lib.HGX_OPT_PUSH_INLINE, 0)
        if gi == 0:
            with pytest.raises(HGXUnsupported):
                snap.set_option(_lib.HGX_OPT_PUSH_INLINE, 1)
        snap.set_option(_lib.HGX_OPT_BFS_BLOCK, 0)
        if gi == 2:
            lt = int(g["subsumes_type"])
            modes = [(False, True, False, False), (False, True, True, False)]
            seeds = np.asarray(g["seeds"], np.int32)
        else:
            modes = K.ALGEN_MODES[::2] if gi == 0 else K.ALGEN_MODES[1::3]
            seeds = rng.integers(0, g["num_atoms"], ns).astype(np.int32)
        for mode in modes:
            check_batch(g, seeds, maxd, mode, lt, snap, orc)
        snap.close()


def test_rows_engine_flag_sets_and_removed_coded_option():
    """The rows engine (HGX_OPT_BFS_BLOCK 0) under three flag sets against the oracle's per-depth sets on
    power-law hubs (heavy chunks), typed links, links targeting links, repeated targets, 300 / 1024 / 2100
    seeds and config 2 at 1%.  HGX_OPT_CODED (coded dense levels, measured slower and removed in round 5)
    accepts only 0."""
    from hypergraphdb_amd import HGXUnsupported, _lib, synth
    rng = np.random.default_rng(321)
    cases = [(synth.hypergraph(3000, 20000, 2, 8, 2.1, 3, seed=31), -1, 3, 1024),
             (synth.hypergraph(3000, 20000, 2, 8, 2.1, 3, seed=32), 1, None, 300),
             (K.random_graph(rng, 1500, 6000, max_arity=12, n_types=3), -1, None, 2100),
             (synth.config2(scale=0.01), -1, 4, 1024)]
    for ci, (g, lt, maxd, ns) in enumerate(cases):
        snap, orc = snapshot(g), oracle(g)
        snap.set_option(_lib.HGX_OPT_CODED, 0)
        if ci == 0:
            for v in (1, 2):
                with pytest.raises(HGXUnsupported):
                    snap.set_option(_lib.HGX_OPT_CODED, v)
        snap.set_option(_lib.HGX_OPT_BFS_BLOCK, 0)
        seeds = rng.integers(0, g["num_atoms"], ns).astype(np.int32)
        for flags in (0x3BE, 0x3BA, 0x1BE):
            snap.set_option(_lib.HGX_OPT_BFS_FLAGS, flags)
            check_batch(g, seeds, maxd, K.ALGEN_MODES[0], lt, snap, orc)


def _all_levels(res):
    return [gpu_levels(res, i) for i in range(res.n_seeds)]


@pytest.mark.parametrize("case", range(6))
def test_workgroup_stage_vs_rows_engine(case):
    """HGX_OPT_BFS_BLOCK: the workgroup-per-seed stage (its seeds' V_d from LDS) + the rows engine on
    the seeds that outgrew it give exactly the rows engine's per-depth sets, counts, depth_of and
    TEPS numerator -- every generator mode, typed links, depth limits 0..4 and unbounded, links
    targeting links, repeated targets, seeds without incidence, duplicate seeds, inline (<= 32) and
    device seed lists, > 4096 seeds (two launches, the second of 4 seeds: inline), and batches where some seeds overflow the
    workgroup (hubs) next to small ones."""
    from hypergraphdb_amd import _lib, bfs_batch, synth
    rng = np.random.default_rng(700 + case)
    if case < 3:
        g = K.random_graph(rng, int(rng.integers(300, 2500)), int(rng.integers(100, 1800)), max_arity=9,
                           link_targets=case != 1, n_types=3)
    elif case < 5:
        g = synth.hypergraph(8000, 9000, 2, 6, 2.1, 2, seed=80 + case)
    else:
        g = synth.config5(scale=0.002, n_sources=300)
    snap = snapshot(g)
    n_seeds = [20, 700, 4100, 300, 1024, 300][case]
    seeds = rng.integers(0, g["num_atoms"], n_seeds).astype(np.int32)
    seeds[-1] = seeds[0]
    mixed = False
    for mi, mode in enumerate(K.ALGEN_MODES):
        lt = [-1, 0, 1, -1, 2, -1][(mi + case) % 6] if case != 5 else int(g["subsumes_type"])
        for maxd in ((None, 0, 2) if case != 2 else (None, 3)):
            res = {}
            for blk in (1, 0):
                snap.set_option(_lib.HGX_OPT_BFS_BLOCK, blk)
                r = bfs_batch(snap, seeds, maxd, gen(snap, mode, lt))
                res[blk] = (r.counts().copy(), _all_levels(r) if case != 2 else None,
                            r.stats()["traversed_edges"], r.stats(accounting=False), r)
            (c1, l1, t1, s1, r1), (c0, l0, t0, s0, r0) = res[1], res[0]
            n = max(c1.shape[1], c0.shape[1])
            pad = lambda c: np.pad(c, ((0, 0), (0, n - c.shape[1])))
            assert np.array_equal(pad(c1), pad(c0)), (case, mi, maxd)
            assert l1 == l0, (case, mi, maxd)
            assert t1 == t0, (case, mi, maxd)
            assert s1["block_seeds"] + s1["block_rerun"] == n_seeds and s0["block_seeds"] == 0
            mixed |= s1["block_seeds"] > s1["block_coop"] and s1["block_rerun"] + s1["block_coop"] > 0
            for i in range(0, n_seeds, max(1, n_seeds // 7)):
                for a in rng.integers(0, g["num_atoms"], 4).tolist() + [int(seeds[i])]:
                    assert r1.depth_of(i, a) == r0.depth_of(i, a), (case, mi, maxd, i, a)
            r1.close()
            r0.close()
    if case in (3, 4):
        assert mixed   # hubs pushed some seeds onto the rows engine next to workgroup seeds
    snap.close()


def test_workgroup_stage_vs_oracle_and_capacity_edges():
    """Seeds whose closure sits just below / above the workgroup's 1534 atoms and 1024-atom levels
    (a path, a star, a binary tree), against the oracle."""
    from hypergraphdb_amd import _lib, bfs_batch
    # star: centre 0 with k leaves as one link each -> level 1 of k atoms
    rows = []
    for k, base in ((1024, 0), (1025, 2000)):
        rows += [[base, base + 1 + j] for j in range(k)]
    # path of 1600 atoms (1599 pairs past the seed: overflows on atom count, not width)
    rows += [[4000 + j, 4001 + j] for j in range(1599)]
    # binary tree of 1535 nodes (1534 past the root)
    rows += [[6000 + j, 6000 + 2 * j + 1, 6000 + 2 * j + 2] for j in range(767)]
    A = 8000
    tgt_off = np.zeros(len(rows) + 1, np.int64)
    tgt_off[1:] = np.cumsum([len(r) for r in rows])
    g = dict(num_atoms=A + len(rows), link_atom=np.arange(A, A + len(rows), dtype=np.int32), tgt_off=tgt_off,
             tgt_idx=np.concatenate(rows).astype(np.int32), link_type=None)
    snap, orc = snapshot(g), oracle(g)
    seeds = np.array([0, 2000, 4000, 4800, 6000, 6001, 7999], np.int32)
    check_batch(g, seeds, None, K.ALGEN_MODES[0], -1, snap, orc)
    check_batch(g, seeds, 5, K.ALGEN_MODES[2], -1, snap, orc)
    r = bfs_batch(snap, seeds, None)
    st = r.stats(accounting=False)
    r.close()
    assert st["block_seeds"] - st["block_coop"] >= 3 and st["block_rerun"] + st["block_coop"] >= 2, st


def test_config5_full_workgroup_stage():
    """Config 5 at full size (5M classes, the bench's 1024 classes): with the workgroup stage on,
    hg.subsumed / hg.subsumes counts and traversed items equal the rows engine's; the big
    hg.subsumed closures go to the rows engine, every hg.subsumes closure stays in a workgroup;
    sampled sets against the oracle."""
    from hypergraphdb_amd import AtomTypeCondition, DefaultALGenerator, _lib, bfs_batch, synth
    g = synth.config5()
    snap, orc = snapshot(g), oracle(g)
    T = g["subsumes_type"]
    for rev in (False, True):
        gen_ = DefaultALGenerator(snap, AtomTypeCondition(T), None, False, True, rev)
        out = {}
        for blk in (1, 0):
            snap.set_option(_lib.HGX_OPT_BFS_BLOCK, blk)
            r = bfs_batch(snap, g["seeds"], None, gen_)
            out[blk] = (r.counts().copy(), r.stats()["traversed_edges"], r.stats(accounting=False), r)
        (c1, t1, s1, r1), (c0, t0, _, r0) = out[1], out[0]
        assert np.array_equal(c1, c0) and t1 == t0, rev
        big = int((c0[:, 1:].sum(1) > 1534).sum())   # closures beyond the workgroup's atoms
        handed = s1["block_rerun"] + s1["block_coop"]   # to the multi-workgroup stage or the rows engine
        assert handed >= big and (handed == 0) == rev, (rev, s1, big)
        for i in (0, 5, 511, 1023):
            lv = orc.bfs_levels(int(g["seeds"][i]), -1, algen(T, False, True, rev, False))
            for d_, exp in enumerate(lv):
                assert np.array_equal(r1.visited(i, d_), exp), (rev, i, d_)
        r1.close()
        r0.close()
    snap.close()


@pytest.mark.parametrize("case", range(5))
def test_multi_workgroup_stage_vs_rows_engine(case):
    """HGX_OPT_BFS_BLOCK 2: a batch of <= 64 seeds straight to the multi-workgroup stage (one persistent
    launch, a grid barrier per level, per-seed visited bitmaps, hub incidence spread over work items)
    gives the rows engine's per-depth sets, counts, depth_of and TEPS numerator in every generator
    mode, typed links, depth limits, duplicate seeds, seeds without incidence; and the bitmaps it
    leaves behind are clean (the next batch on the same graph is exact too)."""
    from hypergraphdb_amd import _lib, bfs_batch, synth
    rng = np.random.default_rng(800 + case)
    if case < 2:
        g = K.random_graph(rng, int(rng.integers(500, 3000)), int(rng.integers(300, 3000)), max_arity=9,
                           link_targets=case == 0, n_types=3)
    elif case < 4:
        g = synth.hypergraph(20000, 40000, 2, 8, 2.1, 3, seed=90 + case)
    else:
        g = synth.config5(scale=0.01, n_sources=64)
    snap = snapshot(g)
    n_seeds = [1, 64, 40, 7, 64][case]
    seeds = (np.asarray(g["seeds"][:n_seeds], np.int32) if case == 4
             else rng.integers(0, g["num_atoms"], n_seeds).astype(np.int32))
    if n_seeds > 2:
        seeds[-1] = seeds[0]
    modes = [(False, True, False, False), (False, True, True, False)] if case == 4 else K.ALGEN_MODES
    for mi, mode in enumerate(modes):
        lt = int(g["subsumes_type"]) if case == 4 else [-1, 0, 1, -1, 2][(mi + case) % 5]
        for maxd in (None, 1, 3):
            res = {}
            for blk in (2, 0):
                snap.set_option(_lib.HGX_OPT_BFS_BLOCK, blk)
                r = bfs_batch(snap, seeds, maxd, gen(snap, mode, lt))
                res[blk] = (r.counts().copy(), _all_levels(r), r.stats()["traversed_edges"],
                            r.stats(accounting=False), r)
            (c2, l2, t2, s2, r2), (c0, l0, t0, s0, r0) = res[2], res[0]
            n = max(c2.shape[1], c0.shape[1])
            pad = lambda c: np.pad(c, ((0, 0), (0, n - c.shape[1])))
            assert s2["block_coop"] == n_seeds, s2
            assert np.array_equal(pad(c2), pad(c0)), (case, mi, maxd)
            assert l2 == l0, (case, mi, maxd)
            assert t2 == t0, (case, mi, maxd)
            for i in range(0, n_seeds, max(1, n_seeds // 5)):
                for a in rng.integers(0, g["num_atoms"], 4).tolist() + [int(seeds[i])]:
                    assert r2.depth_of(i, a) == r0.depth_of(i, a), (case, mi, maxd, i, a)
            r2.close()
            r0.close()
    snap.close()


@pytest.mark.parametrize("blk", (1, 2))
def test_grid_stage_barrier_timeout_falls_back(blk):
    """a grid-stage launch whose barrier times out (its workgroups not all resident in
    time; forced here with a limit of one clock tick, HGX_OPT_CO_TIMEOUT) must not be reported as finished.
    Its seeds rerun on the rows engine with exact results, the fallback is counted (coop_fallbacks), and
    the bitmaps it left are cleared: the next batch on the same graph, with the normal limit, is exact
    and runs on the grid stage.  blk 1: the chained hand-over behind the workgroup stage; blk 2: the
    host-driven launch."""
    from hypergraphdb_amd import AtomTypeCondition, DefaultALGenerator, _lib, bfs_batch, synth
    g = synth.config5(scale=0.05, n_sources=200)
    snap = snapshot(g)
    T = int(g["subsumes_type"])
    gen_ = DefaultALGenerator(snap, AtomTypeCondition(T), None, False, True, False)
    snap.set_option(_lib.HGX_OPT_BFS_BLOCK, 0)
    # the first classes (the root and its first subclasses: closures far beyond a workgroup) + 200 others
    all_seeds = np.concatenate([np.arange(8, dtype=np.int32), np.asarray(g["seeds"], np.int32)])
    ref = bfs_batch(snap, all_seeds, None, gen_)
    c_ref, t_ref = ref.counts().copy(), ref.stats()["traversed_edges"]
    # the seeds whose closure outgrows a workgroup (the grid stage's)
    big = np.nonzero(c_ref[:, 1:].sum(1) > 1534)[0]
    assert 1 <= len(big) <= 64, len(big)
    seeds = all_seeds if blk == 1 else all_seeds[big]
    c_want = c_ref if blk == 1 else c_ref[big]
    lv_want = {i: [ref.visited(int(i), d).copy() for d in range(c_ref.shape[1])] for i in big[:3]}
    ref.close()
    snap.set_option(_lib.HGX_OPT_BFS_BLOCK, blk)
    for limit in (1, 0):
        snap.set_option(_lib.HGX_OPT_CO_TIMEOUT, limit)
        r = bfs_batch(snap, seeds, None, gen_)
        c = r.counts()
        n = max(c.shape[1], c_want.shape[1])
        pad = lambda x: np.pad(x, ((0, 0), (0, n - x.shape[1])))
        assert np.array_equal(pad(c), pad(c_want)), limit
        st = r.stats(accounting=False)
        if limit:
            assert st["coop_fallbacks"] >= 1 and st["block_coop"] == 0, st
        else:
            assert st["coop_fallbacks"] == 0 and st["block_coop"] == len(big), st
        for i in big[:3]:
            j = int(i) if blk == 1 else int(np.nonzero(big == i)[0][0])
            for d, exp in enumerate(lv_want[i]):
                assert np.array_equal(r.visited(j, d), exp), (limit, int(i), d)
        r.close()
    if blk == 1:
        r = bfs_batch(snap, seeds, None, gen_)
        assert r.stats()["traversed_edges"] == t_ref
        r.close()
    snap.close()


@pytest.mark.parametrize("case", ("config5", "hubs"))
def test_grid_stage_stress(case):
    """VERDICT r4 'do this' 8: the grid stage (HGX_OPT_BFS_BLOCK 2, every seed of the batch in one
    persistent launch) on the 64 largest hg.subsumed closures of the full config-5 bench batch (2K-101K
    atoms over ~21 levels), and on 64 hub seeds of a power-law graph in the symmetric mode (levels of
    tens of thousands of atoms, hub incidence split over many work items), against the rows engine
    (counts, sets, TEPS numerator) and oracle samples.  Every cross-workgroup access of hgx_bfs_coop is
    an agent-scope atomic (co_put / co_get, atomicOr, the counters), the precondition of its light
    barrier; a plain store there would show up here as a wrong set."""
    from hypergraphdb_amd import AtomTypeCondition, DefaultALGenerator, _lib, bfs_batch, synth
    if case == "config5":
        g = synth.config5()
        snap, orc = snapshot(g), oracle(g)
        T = int(g["subsumes_type"])
        gen_ = DefaultALGenerator(snap, AtomTypeCondition(T), None, False, True, False)
        opts = algen(T, False, True, False, False)
        snap.set_option(_lib.HGX_OPT_BFS_BLOCK, 0)
        r = bfs_batch(snap, g["seeds"], None, gen_)
        sizes = r.counts()[:, 1:].sum(1)
        r.close()
        seeds = np.asarray(g["seeds"], np.int32)[np.argsort(-sizes, kind="stable")[:64]]
        maxd = None
    else:
        g = synth.hypergraph(60000, 120000, 2, 8, 2.1, 3, seed=77)
        snap, orc = snapshot(g), oracle(g)
        gen_ = None
        opts = None
        deg = np.bincount(np.asarray(g["tgt_idx"]), minlength=g["num_atoms"])
        seeds = np.argsort(-deg, kind="stable")[:64].astype(np.int32)
        maxd = 2
    res = {}
    for blk in (2, 0):
        snap.set_option(_lib.HGX_OPT_BFS_BLOCK, blk)
        r = bfs_batch(snap, seeds, maxd, gen_)
        res[blk] = (r.counts().copy(), r.stats()["traversed_edges"], r.stats(accounting=False), r)
    (c2, t2, s2, r2), (c0, t0, _, r0) = res[2], res[0]
    assert s2["block_coop"] == 64 and s2["coop_fallbacks"] == 0, {k: s2[k] for k in ("block_coop", "coop_fallbacks", "block_rerun", "block_seeds")}
    n = max(c2.shape[1], c0.shape[1])
    pad = lambda c: np.pad(c, ((0, 0), (0, n - c.shape[1])))
    assert np.array_equal(pad(c2), pad(c0)) and t2 == t0
    for i in range(64):
        for d in range(n):
            assert np.array_equal(r2.visited(i, d), r0.visited(i, d)), (case, i, d)
    for i in (0, 31, 63):
        lv = orc.bfs_levels(int(seeds[i]), -1 if maxd is None else maxd, opts)
        for d, exp in enumerate(lv):
            assert np.array_equal(r2.visited(i, d), exp), (case, i, d)
    r2.close()
    r0.close()
    snap.close()
