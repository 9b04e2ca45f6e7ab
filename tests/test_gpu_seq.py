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
