"""GPU parity: order-exact traversal (hgx_bfs_sequence) -- the exact (link, atom) sequence of
HGBreadthFirstTraversal.next() (C/algorithms/HGBreadthFirstTraversal.java:49-66,143-156) against
the golden fixtures and the oracle, bit-exact including FIFO order and discovering links."""
import json
import os

import numpy as np
import pytest

import kat_graphs as K
from oracle_ctypes import algen
from test_gpu_bfs import gen, oracle, snapshot

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def check_seq(g, seeds, maxd, mode, lt=-1, snap=None, orc=None):
    from hypergraphdb_amd import bfs_sequence
    snap = snap or snapshot(g)
    orc = orc or oracle(g)
    res = bfs_sequence(snap, seeds, maxd, gen(snap, mode, lt))
    trav = 0
    for i, s in enumerate(seeds):
        l, a, d, tr = orc.bfs(int(s), -1 if maxd is None else maxd, algen(lt, *mode))
        gl, ga, gd = res.pairs(i)
        assert np.array_equal(ga, a), (i, s, mode, maxd, lt, "atoms")
        assert np.array_equal(gl, l), (i, s, mode, maxd, lt, "links")
        assert np.array_equal(gd, d), (i, s, mode, maxd, lt, "dists")
        trav += tr
    assert res.traversed_edges == float(trav)
    return res


def test_kat_fixture_sequences_every_seed_every_mode():
    from hypergraphdb_amd import bfs_sequence
    with open(os.path.join(GOLD, "kat.json")) as f:
        kat = json.load(f)
    for name, e in kat.items():
        g = {k: np.asarray(v) if isinstance(v, list) else v for k, v in e.items() if k not in ("bfs", "incidence")}
        snap = snapshot(g)
        seeds = list(range(g["num_atoms"]))
        for mi, mode in enumerate(K.ALGEN_MODES):
            for maxd in (None, 1, 2):
                res = bfs_sequence(snap, seeds, maxd, gen(snap, mode))
                for s in seeds:
                    exp = [tuple(x) for x in e["bfs"][f"{s}/{mi}/{maxd}"]]
                    got = list(zip(*(x.tolist() for x in res.pairs(s))))
                    assert got == exp, (name, s, mode, maxd)
        snap.close()


def test_random_fixture_sequences():
    from hypergraphdb_amd import bfs_sequence
    d = np.load(os.path.join(GOLD, "random_small.npz"))
    gi = 0
    while f"g{gi}_A" in d:
        g = dict(num_atoms=int(d[f"g{gi}_A"][0]), link_atom=d[f"g{gi}_link_atom"], tgt_off=d[f"g{gi}_tgt_off"],
                 tgt_idx=d[f"g{gi}_tgt_idx"], link_type=d[f"g{gi}_link_type"])
        snap = snapshot(g)
        pos = 0
        seq_all = [tuple(x) for x in d[f"g{gi}_bfs_seq"].tolist()]
        for seed, mi, lt, maxd, n in d[f"g{gi}_bfs_keys"].tolist():
            res = bfs_sequence(snap, [seed], None if maxd < 0 else maxd, gen(snap, K.ALGEN_MODES[mi], lt))
            got = list(zip(*(x.tolist() for x in res.pairs(0))))
            assert got == seq_all[pos:pos + n], (gi, seed, mi, lt, maxd)
            pos += n
        snap.close()
        gi += 1


@pytest.mark.parametrize("case", range(6))
def test_random_graphs_all_modes(case):
    """Links targeting links, repeated targets, arity 0/1 links, typed predicates, duplicate seeds."""
    rng = np.random.default_rng(900 + case)
    g = K.random_graph(rng, int(rng.integers(200, 1500)), int(rng.integers(200, 2500)), max_arity=7,
                       link_targets=case % 2 == 0, n_types=3)
    mode = K.ALGEN_MODES[case % len(K.ALGEN_MODES)]
    seeds = rng.integers(0, g["num_atoms"], [1, 5, 64, 100, 130, 40][case]).astype(np.int32)
    seeds[-1] = seeds[0]
    lt = [-1, 0, 1, -1, 2, -1][case]
    maxd = [None, 2, 3, None, 1, 4][case]
    check_seq(g, seeds, maxd, mode, lt)


def test_ragged_last_launch():
    """1024 + 5 seeds: the workgroup engine's second launch holds 5 seeds, passed in the kernel
    arguments while the first launch reads a device list."""
    rng = np.random.default_rng(77)
    g = K.random_graph(rng, 600, 900, max_arity=5, n_types=2)
    seeds = rng.integers(0, g["num_atoms"], 1029).astype(np.int32)
    check_seq(g, seeds, None, K.ALGEN_MODES[0])
    check_seq(g, seeds, 2, K.ALGEN_MODES[3], 1)


def test_power_law_hubs_and_chunking():
    """Hubs (long incidence rows spanning many expand tiles) and a 1 MiB working-set budget that
    forces the seeds through several chunks."""
    from hypergraphdb_amd import _lib, synth
    g = synth.hypergraph(3000, 20000, 2, 8, 2.1, 3, seed=21)
    snap, orc = snapshot(g), oracle(g)
    seeds = np.concatenate([np.arange(4), np.arange(2950, 3000)]).astype(np.int32)
    check_seq(g, seeds, 3, K.ALGEN_MODES[0], -1, snap, orc)
    snap.set_option(_lib.HGX_OPT_SEQ_BUDGET, 1 << 20)
    check_seq(g, seeds, None, K.ALGEN_MODES[1], 2, snap, orc)
    check_seq(g, seeds, None, K.ALGEN_MODES[4], -1, snap, orc)


def test_config1_sequences_sampled_seeds():
    from hypergraphdb_amd import synth
    g = synth.config1()
    check_seq(g, g["seeds"][:16], 3, K.ALGEN_MODES[0])


def test_traversal_iterator_matches_reference_order():
    from hypergraphdb_amd import DefaultALGenerator, HGBreadthFirstTraversal
    rng = np.random.default_rng(5)
    g = K.random_graph(rng, 400, 700, max_arity=6, n_types=2)
    snap, orc = snapshot(g), oracle(g)
    start = int(g["tgt_idx"][0])
    tr = HGBreadthFirstTraversal(start, DefaultALGenerator(snap), 3)
    assert tr.isVisited(start)                      # examined.put(start, TRUE) (:42-46)
    l, a, d, _ = orc.bfs(start, 3)
    got = []
    while tr.hasNext():
        link, atom = tr.next()
        assert tr.isVisited(atom)
        got.append((link, atom, tr.distance()))
    assert got == list(zip(l.tolist(), a.tolist(), d.tolist()))
    assert tr.next() is None
    tr.reset()
    assert tr.hasNext() == (len(a) > 0)


def _seq(snap, seeds, maxd, g_, engine):
    from hypergraphdb_amd import _lib, bfs_sequence
    snap.set_option(_lib.HGX_OPT_SEQ_ENGINE, engine)
    try:
        return bfs_sequence(snap, seeds, maxd, g_)
    finally:
        snap.set_option(_lib.HGX_OPT_SEQ_ENGINE, 0)


@pytest.mark.parametrize("case", range(4))
def test_workgroup_and_level_engines_agree(case):
    """The workgroup-per-seed engine (default), the level-synchronous hgx_ls_* engine (2) and the
    round-1 key-array engine (1) return identical sequences, links, distances and traversal counts --
    over graphs whose closures stay inside one workgroup and graphs whose hubs push some seeds over its
    2046 pairs (those rerun on the level-synchronous engine)."""
    from hypergraphdb_amd import synth
    rng = np.random.default_rng(40 + case)
    if case < 2:
        g = K.random_graph(rng, 3000, 2000, max_arity=9, link_targets=True, n_types=3)
    else:
        g = synth.hypergraph(6000, 9000, 2, 6, 2.1, 2, seed=70 + case)
    snap = snapshot(g)
    seeds = rng.integers(0, g["num_atoms"], 300).astype(np.int32)
    for mi, mode in enumerate(K.ALGEN_MODES):
        lt = [-1, 0, 1][mi % 3] if case % 2 == 0 else -1
        for maxd in (None, 2):
            a = _seq(snap, seeds, maxd, gen(snap, mode, lt), 0)
            for eng in (1, 2):
                b = _seq(snap, seeds, maxd, gen(snap, mode, lt), eng)
                assert np.array_equal(a.offsets, b.offsets), (case, mi, maxd, eng)
                assert np.array_equal(a.atoms, b.atoms) and np.array_equal(a.links, b.links), (case, mi, maxd, eng)
                assert np.array_equal(a.dists, b.dists), (case, mi, maxd, eng)
                assert a.traversed_edges == b.traversed_edges and a.n_levels == b.n_levels, eng
    snap.close()


def test_workgroup_engine_overflow_mixed_with_small_seeds_vs_oracle():
    """A batch mixing seeds whose traversal exceeds the workgroup's pairs (hub neighbourhoods) with
    tiny ones, checked seed by seed against the oracle."""
    from hypergraphdb_amd import synth
    g = synth.hypergraph(20000, 30000, 2, 5, 2.0, 1, seed=5)
    snap, orc = snapshot(g), oracle(g)
    deg = np.diff(np.searchsorted(np.sort(g["tgt_idx"]), np.arange(g["num_atoms"] + 1)))
    hubs = np.argsort(-deg)[:3].astype(np.int32)
    seeds = np.concatenate([hubs, np.arange(19990, 20000, dtype=np.int32), hubs[:1]])
    res = check_seq(g, seeds, 3, K.ALGEN_MODES[0], -1, snap, orc)
    assert (np.diff(res.offsets) > 2046).any() and (np.diff(res.offsets) <= 2046).any()


def test_config5_closures_sequence_vs_oracle():
    """Config 5 (5M classes, full size): hg.subsumed / hg.subsumes as order-exact sequences for 128
    classes of the bench's 1024 against the oracle, pair by pair; the batch of 1024 equals the
    concatenation of single-seed calls (the drop-in issues one traversal per HGGpuTraversal)."""
    from hypergraphdb_amd import AtomTypeCondition, DefaultALGenerator, bfs_sequence, synth
    g = synth.config5()
    snap, orc = snapshot(g), oracle(g)
    T = g["subsumes_type"]
    for rev in (False, True):
        gen_ = DefaultALGenerator(snap, AtomTypeCondition(T), None, False, True, rev)
        res = bfs_sequence(snap, g["seeds"], None, gen_)
        for i in range(0, 1024, 8):
            l_, a, d, _ = orc.bfs(int(g["seeds"][i]), -1, algen(T, False, True, rev, False))
            gl, ga, gd = res.pairs(i)
            assert np.array_equal(ga, a) and np.array_equal(gl, l_) and np.array_equal(gd, d), (rev, i)
        for i in (0, 1, 511, 1023):
            one = bfs_sequence(snap, g["seeds"][i:i + 1], None, gen_)
            assert all(np.array_equal(x, y) for x, y in zip(one.pairs(0), res.pairs(i))), (rev, i)
    snap.close()


def test_level_engine_capacity_growth_and_depth_limits():
    """The level-synchronous engine grows its capacities (discoveries, bitmap words, tiles, runs)
    from small starting values on a graph whose levels exceed them, then stays exact; every depth
    limit 0..4 and unbounded, against the oracle."""
    from hypergraphdb_amd import _lib, synth
    g = synth.hypergraph(30000, 60000, 2, 6, 2.0, 1, seed=13)
    snap, orc = snapshot(g), oracle(g)
    snap.set_option(_lib.HGX_OPT_SEQ_SMALL, 1)
    snap.set_option(_lib.HGX_OPT_SEQ_ENGINE, 2)
    seeds = np.array([0, 1, 2, 29999, 15000, 0], np.int32)
    for maxd in (0, 1, 2, 3, 4, None):
        check_seq(g, seeds, maxd, K.ALGEN_MODES[maxd % 3 if maxd else 0], -1, snap, orc)
    snap.set_option(_lib.HGX_OPT_SEQ_ENGINE, 0)


# the level engine's test options (hgx_set_option; the library reads no tuning knob from the environment)
SEQ_OPTS = {"pull": "HGX_OPT_SEQ_PULL", "small": "HGX_OPT_SEQ_SMALL", "tlimit": "HGX_OPT_SEQ_TLIMIT",
            "pack_min": "HGX_OPT_SEQ_PACK_MIN"}
SEQ_DEFAULTS = {"pull": 1, "small": 0, "tlimit": 0, "pack_min": 0}


def _seq_opts(snap, seeds, maxd, g_, opts):
    """hgx_bfs_sequence on the level-synchronous engine alone (HGX_OPT_SEQ_ENGINE 2) under the given level
    engine options (restored to the defaults afterwards)."""
    from hypergraphdb_amd import _lib, bfs_sequence
    for k, v in opts.items():
        snap.set_option(getattr(_lib, SEQ_OPTS[k]), int(v))
    snap.set_option(_lib.HGX_OPT_SEQ_ENGINE, 2)
    try:
        return bfs_sequence(snap, seeds, maxd, g_)
    finally:
        snap.set_option(_lib.HGX_OPT_SEQ_ENGINE, 0)
        for k in opts:
            snap.set_option(getattr(_lib, SEQ_OPTS[k]), SEQ_DEFAULTS[k])


@pytest.mark.parametrize("case", range(5))
def test_level_engine_pull_and_push_levels_agree(case):
    """Round 5: the level engine without a per-seed key array.  Every level pushed (HGX_OPT_SEQ_PULL 0: the
    level hash), every level pulled (2: frontier rows, union bitmap, pin index, per-seed minima in LDS;
    heavy atoms by 4096-entry chunks), and the default choice by width (1) give the oracle's exact
    sequences -- links, atoms, distances, traversed items -- in every generator mode, with typed links,
    links targeting links, repeated targets, duplicate seeds, > 64 seeds (several row words) and hubs
    above 512 incidences (the pull's heavy chunks); starting capacities tiny (HGX_OPT_SEQ_SMALL) in case 4."""
    from hypergraphdb_amd import synth
    rng = np.random.default_rng(950 + case)
    if case < 2:
        g = K.random_graph(rng, int(rng.integers(800, 2500)), int(rng.integers(1500, 3000)), max_arity=9,
                           link_targets=case == 0, n_types=3)
    else:
        g = synth.hypergraph(3000, 20000, 2, 8, 2.1, 3, seed=60 + case)
    snap, orc = snapshot(g), oracle(g)
    n_seeds = [40, 70, 130, 64, 300][case]
    seeds = rng.integers(0, g["num_atoms"], n_seeds).astype(np.int32)
    seeds[-1] = seeds[0]
    extra = {"small": 1} if case == 4 else {}
    pulled = 0
    for mi, mode in enumerate(K.ALGEN_MODES):
        if case >= 2 and mi % 3:
            continue
        lt = [-1, 0, 1][(mi + case) % 3]
        for maxd in ((None, 2) if case != 3 else (3,)):
            outs = {}
            for pull in (0, 2, 1):
                outs[pull] = _seq_opts(snap, seeds, maxd, gen(snap, mode, lt), dict(extra, pull=pull))
            a = outs[0]
            for pull in (2, 1):
                b = outs[pull]
                assert np.array_equal(a.offsets, b.offsets), (case, mi, maxd, pull)
                assert np.array_equal(a.atoms, b.atoms) and np.array_equal(a.links, b.links), (case, mi, maxd, pull)
                assert np.array_equal(a.dists, b.dists) and a.traversed_edges == b.traversed_edges, (case, mi, maxd)
            assert outs[0].pull_levels == 0 and outs[2].pull_levels >= 1, (outs[0].pull_levels, outs[2].pull_levels)
            pulled += outs[2].pull_levels
            for i in range(0, n_seeds, max(1, n_seeds // 6)):
                l_, at, d, _ = orc.bfs(int(seeds[i]), -1 if maxd is None else maxd, algen(lt, *mode))
                gl, ga, gd = a.pairs(i)
                assert np.array_equal(ga, at) and np.array_equal(gl, l_) and np.array_equal(gd, d), (case, mi, maxd, i)
    assert pulled > 0
    snap.close()


@pytest.mark.parametrize("case", range(3))
def test_level_engine_packed_transfer(case):
    """Round 5: large levels go to the host packed (atoms, run-start bits, the links of run starts, block
    run counts; HGX_OPT_SEQ_PACK_MIN, default 2^20 pairs).  Packing every level (1) gives the unpacked engine's
    exact sequences and the oracle's, through the whole-result readout and through ranged reads whose
    windows start anywhere (inside a run of one link, at a rank-part boundary); one seed, repeated links and
    > 64 seeds included."""
    import ctypes as C
    from hypergraphdb_amd import synth
    from hypergraphdb_amd._lib import check, lib, ptr
    rng = np.random.default_rng(970 + case)
    g = synth.hypergraph(3000, 20000, 2, 8, 2.1, 3, seed=70 + case) if case else \
        K.random_graph(rng, 2000, 2500, max_arity=9, link_targets=True, n_types=2)
    snap, orc = snapshot(g), oracle(g)
    seeds = rng.integers(0, g["num_atoms"], [1, 70, 130][case]).astype(np.int32)
    for mi, mode in enumerate(K.ALGEN_MODES[:3]):
        for maxd in (2, None):
            gn = gen(snap, mode, -1)
            a = _seq_opts(snap, seeds, maxd, gn, {"pack_min": 1 << 40})
            b = _seq_opts(snap, seeds, maxd, gn, {"pack_min": 1})
            assert np.array_equal(a.offsets, b.offsets), (case, mi, maxd)
            assert np.array_equal(a.atoms, b.atoms) and np.array_equal(a.links, b.links), (case, mi, maxd)
            assert np.array_equal(a.dists, b.dists) and a.traversed_edges == b.traversed_edges, (case, mi, maxd)
            for i in range(0, len(seeds), max(1, len(seeds) // 4)):
                l_, at, d, _ = orc.bfs(int(seeds[i]), -1 if maxd is None else maxd, algen(-1, *mode))
                gl, ga, gd = b.pairs(i)
                assert np.array_equal(ga, at) and np.array_equal(gl, l_) and np.array_equal(gd, d), (case, mi, maxd, i)
    # ranged reads of a packed result: every start position of a sample, short and long windows
    from hypergraphdb_amd import _lib
    snap.set_option(_lib.HGX_OPT_SEQ_PACK_MIN, 1)
    snap.set_option(_lib.HGX_OPT_SEQ_ENGINE, 2)
    h = C.c_void_p()
    try:
        opts = gen(snap, K.ALGEN_MODES[0], -1).options()
        check(lib().hgx_bfs_sequence(snap.handle, ptr(seeds), len(seeds), -1, C.byref(opts), C.byref(h)))
    finally:
        snap.set_option(_lib.HGX_OPT_SEQ_ENGINE, 0)
        snap.set_option(_lib.HGX_OPT_SEQ_PACK_MIN, 0)
    try:
        ns, npairs, nl = C.c_int32(), C.c_int64(), C.c_int32()
        check(lib().hgx_seq_result_info(h, C.byref(ns), C.byref(npairs), C.byref(nl)))
        n = npairs.value
        links, atoms, dists = (np.empty(max(n, 1), np.int32) for _ in range(3))
        check(lib().hgx_seq_result_pairs(h, ptr(links), ptr(atoms), ptr(dists)))
        vp = lambda x: C.c_void_p(ptr(x))
        starts = sorted(set(rng.integers(0, max(n, 1), 200).tolist() + [0, max(n - 1, 0)]))
        for first in starts:
            for win in (1, 7, 700):
                wl, wa, wd = (np.empty(win, np.int32) for _ in range(3))
                got = C.c_int64()
                check(lib().hgx_seq_result_pairs_range(h, C.c_int64(first), C.c_int64(win), vp(wl), vp(wa), vp(wd),
                                                       C.byref(got)))
                k = got.value
                assert k == min(win, n - first)
                assert np.array_equal(wl[:k], links[first:first + k]), (case, first, win)
                assert np.array_equal(wa[:k], atoms[first:first + k]) and np.array_equal(wd[:k], dists[first:first + k])
    finally:
        lib().hgx_seq_result_free(h)
    snap.close()


def test_level_engine_results_outlive_later_calls():
    """A result's pair copies may still run when hgx_bfs_sequence returns (hgx.h): its readers wait per rank part,
    its free waits for every copy, and a later call on the same graph is ordered after them.  With every level
    packed (HGX_OPT_SEQ_PACK_MIN 1) on the level engine (HGX_OPT_SEQ_ENGINE 2): result A is held while call B runs
    on the same graph (its scratch and the pooled host buffers reused), result D is freed unread and call C
    follows at once; A's stats are read before its pairs, A is read by ranges before it is read whole, and A, B
    and C are the oracle's exact sequences (links, atoms, distances, traversed items)."""
    import ctypes as C
    from hypergraphdb_amd import _lib, synth
    from hypergraphdb_amd._lib import check, lib, ptr
    g = synth.hypergraph(3000, 20000, 2, 8, 2.1, 3, seed=75)
    snap, orc = snapshot(g), oracle(g)
    rng = np.random.default_rng(975)
    sa = rng.integers(0, g["num_atoms"], 70).astype(np.int32)
    sb = rng.integers(0, g["num_atoms"], 130).astype(np.int32)
    sd = sb[::-1].copy()
    sc = rng.integers(0, g["num_atoms"], 33).astype(np.int32)
    mode = K.ALGEN_MODES[0]
    opts = gen(snap, mode, -1).options()

    def call(seeds, maxd):
        h = C.c_void_p()
        check(lib().hgx_bfs_sequence(snap.handle, ptr(seeds), len(seeds), maxd, C.byref(opts), C.byref(h)))
        return h

    def read_whole(h, n_seeds):
        ns, npairs, nl = C.c_int32(), C.c_int64(), C.c_int32()
        check(lib().hgx_seq_result_info(h, C.byref(ns), C.byref(npairs), C.byref(nl)))
        assert ns.value == n_seeds
        off = np.zeros(n_seeds + 1, np.int64)
        check(lib().hgx_seq_result_offsets(h, ptr(off)))
        n = npairs.value
        links, atoms, dists = (np.empty(max(n, 1), np.int32) for _ in range(3))
        check(lib().hgx_seq_result_pairs(h, ptr(links), ptr(atoms), ptr(dists)))
        return off, links[:n], atoms[:n], dists[:n]

    def vs_oracle(seeds, maxd, off, links, atoms, dists):
        trav = 0
        for i, s in enumerate(seeds):
            l_, at, d, tr = orc.bfs(int(s), maxd, algen(-1, *mode))
            b, e = off[i], off[i + 1]
            assert np.array_equal(atoms[b:e], at) and np.array_equal(links[b:e], l_), (i, s, maxd)
            assert np.array_equal(dists[b:e], d), (i, s, maxd)
            trav += tr
        return trav

    snap.set_option(_lib.HGX_OPT_SEQ_PACK_MIN, 1)
    snap.set_option(_lib.HGX_OPT_SEQ_ENGINE, 2)
    held = []
    try:
        ha = call(sa, 3)
        held.append(ha)
        hb = call(sb, 2)   # A unread: B reuses the graph's scratch behind A's copies
        held.append(hb)
        hd = call(sd, 3)
        lib().hgx_seq_result_free(hd)   # freed unread: its buffers go back to the pool after its copies
        hc = call(sc, -1)
        held.append(hc)
        # A: stats first (the lazy timing read), then ranged windows, then the whole readout
        ms, tr = C.c_double(), C.c_double()
        check(lib().hgx_seq_result_stats(ha, C.byref(ms), C.byref(tr)))
        ml, bl, pl = C.c_double(), C.c_double(), C.c_int64()
        check(lib().hgx_seq_result_level_stats(ha, C.byref(ml), C.byref(bl), C.byref(pl)))
        ns, npairs, nl = C.c_int32(), C.c_int64(), C.c_int32()
        check(lib().hgx_seq_result_info(ha, C.byref(ns), C.byref(npairs), C.byref(nl)))
        n = npairs.value
        assert n > 1000
        vp = lambda x: C.c_void_p(ptr(x))
        windows = {}
        for first in sorted(set(rng.integers(0, n, 40).tolist() + [0, n - 1])):
            wl, wa, wd = (np.empty(300, np.int32) for _ in range(3))
            got = C.c_int64()
            check(lib().hgx_seq_result_pairs_range(ha, C.c_int64(first), C.c_int64(300), vp(wl), vp(wa), vp(wd),
                                                   C.byref(got)))
            k = got.value
            assert k == min(300, n - first)
            windows[first] = (wl[:k].copy(), wa[:k].copy(), wd[:k].copy())
        ra = read_whole(ha, len(sa))
        for first, (wl, wa, wd) in windows.items():
            k = len(wl)
            assert np.array_equal(wl, ra[1][first:first + k]) and np.array_equal(wa, ra[2][first:first + k]), first
            assert np.array_equal(wd, ra[3][first:first + k]), first
        assert vs_oracle(sa, 3, *ra) == tr.value
        vs_oracle(sb, 2, *read_whole(hb, len(sb)))
        vs_oracle(sc, -1, *read_whole(hc, len(sc)))
    finally:
        for h in held:
            lib().hgx_seq_result_free(h)
        snap.set_option(_lib.HGX_OPT_SEQ_ENGINE, 0)
        snap.set_option(_lib.HGX_OPT_SEQ_PACK_MIN, 0)
    snap.close()


def test_level_engine_chunk_split_on_wide_keys():
    """A level whose stream keys do not fit 32 bits splits the chunk (HGX_OPT_SEQ_TLIMIT lowers the limit to
    force it down to single seeds; a single seed that still does not fit runs on the key-array engine):
    the sequences stay the oracle's."""
    from hypergraphdb_amd import synth
    g = synth.hypergraph(3000, 20000, 2, 8, 2.1, 3, seed=61)
    snap, orc = snapshot(g), oracle(g)
    deg = np.bincount(np.asarray(g["tgt_idx"]), minlength=g["num_atoms"])
    seeds = np.concatenate([np.argsort(-deg)[:4], np.arange(100, 120)]).astype(np.int32)
    for lim in (2000, 200000):
        res = _seq_opts(snap, seeds, 3, gen(snap, K.ALGEN_MODES[0]), {"tlimit": lim})
        for i in range(len(seeds)):
            l_, at, d, _ = orc.bfs(int(seeds[i]), 3)
            gl, ga, gd = res.pairs(i)
            assert np.array_equal(ga, at) and np.array_equal(gl, l_) and np.array_equal(gd, d), (lim, i)
    snap.close()


@pytest.mark.parametrize("case", range(4))
def test_order_exact_grid_stage_vs_oracle(case):
    """Round 5: the seeds the order-exact workgroup engine hands back (more than 2046 pairs) run in one
    persistent multi-workgroup launch (hgx_seq_coop: level hash, key-space bitmap ranks, a wave per
    bitmap word) when the generator has a yield adjacency.  Exact against the oracle pair by pair (links,
    atoms, distances, traversed items): config-5 closures at 5% scale (the root classes: 12K-250K-atom
    closures over ~20 levels) in both directions with depth limits, a typed power-law graph, and the
    forced barrier timeout (HGX_OPT_CO_TIMEOUT 1: the stage must fall back to the level engine, still exact,
    and leave its bitmaps clean for the next call)."""
    from hypergraphdb_amd import AtomTypeCondition, DefaultALGenerator, _lib, bfs_batch, bfs_sequence, synth
    if case < 3:
        g = synth.config5(scale=0.05, n_sources=40)
        T = int(g["subsumes_type"])
        rev = case == 1
        snap, orc = snapshot(g), oracle(g)
        gen_ = DefaultALGenerator(snap, AtomTypeCondition(T), None, False, True, rev)
        opts = algen(T, False, True, rev, False)
        # classes whose closure outgrows the workgroup engine (> 2046 pairs) but stays below the stage's
        # per-level key space, picked from the set engine's closure sizes, next to small ones
        cand = np.concatenate([np.arange(4000, dtype=np.int32), np.asarray(g["seeds"], np.int32)])
        r = bfs_batch(snap, cand, None, gen_)
        size = r.counts()[:, 1:].sum(1)
        r.close()
        big = cand[(size > 2100) & (size < 30000)][:8]
        assert len(big) >= 1 or rev, size.max()
        seeds = np.concatenate([big, np.asarray(g["seeds"], np.int32)]).astype(np.int32)
        maxds = (None, 3) if case < 2 else (None,)
    else:
        g = synth.hypergraph(6000, 30000, 2, 6, 2.1, 3, seed=88)
        snap, orc = snapshot(g), oracle(g)
        gen_ = gen(snap, K.ALGEN_MODES[1], -1)   # an ordered mode: the yield adjacency exists
        opts = algen(-1, *K.ALGEN_MODES[1])
        cand = np.arange(0, 6000, 7, dtype=np.int32)
        r = bfs_batch(snap, cand, None, gen_)
        size = r.counts()[:, 1:].sum(1)
        r.close()
        big = cand[(size > 2100) & (size < 20000)][:6]
        assert len(big) >= 1, size.max()
        seeds = np.concatenate([big, np.arange(5990, 6000, dtype=np.int32)]).astype(np.int32)
        maxds = (None, 2)
    for maxd in maxds:
        for attempt in ((1, 0) if case == 2 else (0,)):
            snap.set_option(_lib.HGX_OPT_CO_TIMEOUT, 1 if attempt else 0)
            try:
                res = bfs_sequence(snap, seeds, maxd, gen_)
            finally:
                snap.set_option(_lib.HGX_OPT_CO_TIMEOUT, 0)
            trav = 0
            for i, s in enumerate(seeds):
                l_, a, d, tr = orc.bfs(int(s), -1 if maxd is None else maxd, opts)
                gl, ga, gd = res.pairs(i)
                assert np.array_equal(ga, a) and np.array_equal(gl, l_) and np.array_equal(gd, d), (case, maxd, i)
                trav += tr
            assert res.traversed_edges == float(trav)
            if attempt:
                assert res.n_coop == 0 and res.n_level >= 1, (res.n_coop, res.n_level)
            elif case in (0, 2) and maxd is None:   # (hg.subsumes closures stay inside the workgroup engine;
                # case 3's wide levels exceed the stage's key space: the level engine takes them)
                assert res.n_coop >= 1 and res.n_coop == res.n_level, (res.n_coop, res.n_level)
    snap.close()
