"""GPU parity of the snapshot on disk and batched store updates: a graph opened from a .hgcsr file
(hgx_graph_open) and a graph after hgx_graph_update answer BFS batches, incidence reads and pattern
queries exactly as the oracle does on the same rows."""
import numpy as np
import pytest

import kat_graphs as K
from oracle_ctypes import OracleGraph
from test_gpu_bfs import check_batch

pytestmark = pytest.mark.gpu


def oracle(g):
    return OracleGraph(g["num_atoms"], np.asarray(g["link_atom"], np.int32), np.asarray(g["tgt_off"], np.int64),
                       np.asarray(g["tgt_idx"], np.int32), np.asarray(g["link_type"], np.int32))


def random_queries(rng, g, n):
    qs = []
    for _ in range(n):
        t = int(rng.integers(-1, 3))
        inc = [int(x) for x in rng.integers(0, g["num_atoms"], int(rng.integers(1, 3)))]
        m = int(rng.integers(-1, 4))
        pat = None if m < 0 else tuple(int(x) if rng.random() < 0.7 else -1
                                       for x in rng.integers(0, g["num_atoms"], m))
        qs.append((t, inc, pat))
    return qs


def check_all(snap, g, rng, modes=((True, True, False, False), (False, True, False, False),
                                   (True, True, True, True))):
    from hypergraphdb_amd import pattern_batch
    orc = oracle(g)
    seeds = rng.choice(g["num_atoms"], min(64, g["num_atoms"]), replace=False).astype(np.int32)
    for mode in modes:
        check_batch(g, seeds, None, mode, snap=snap, orc=orc)
        check_batch(g, seeds, 2, mode, lt=1, snap=snap, orc=orc)
    for a in range(g["num_atoms"]):
        assert snap.incidence(a).tolist() == orc.incidence(a).tolist(), a
    qs = random_queries(rng, g, 500)
    r = pattern_batch(snap, qs)
    for q, (t, inc, pat) in enumerate(qs):
        assert r[q].tolist() == orc.and_query(t, inc, pat).tolist(), qs[q]


def test_open_matches_create(tmp_path):
    from hypergraphdb_amd import HyperGraphSnapshot, write_snapshot
    rng = np.random.default_rng(70)
    g = K.random_graph(rng, 300, 900, max_arity=6)
    p = str(tmp_path / "g.hgcsr")
    write_snapshot(p, g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    snap = HyperGraphSnapshot.open(p)
    assert snap.A == g["num_atoms"] and snap.M == len(g["link_atom"])
    np.testing.assert_array_equal(snap.tgt_idx, g["tgt_idx"])
    check_all(snap, g, rng)
    snap.close()


def test_save_open_device_only(tmp_path):
    """A device-authoritative snapshot (keep_host=False) saved from the device and re-opened."""
    from hypergraphdb_amd import HyperGraphSnapshot, read_snapshot
    rng = np.random.default_rng(71)
    g = K.random_graph(rng, 200, 700, max_arity=5, link_targets=False)
    s0 = HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"],
                            keep_host=False)
    p = str(tmp_path / "d.hgcsr")
    s0.save(p)
    f = read_snapshot(p)
    for k in ("link_atom", "tgt_off", "tgt_idx", "link_type"):
        np.testing.assert_array_equal(f[k], g[k], err_msg=k)
    s1 = HyperGraphSnapshot.open(p, keep_host=False)
    assert s1.tgt_idx is None and s1.num_incidences == s0.num_incidences
    check_all(s1, g, rng)
    s0.close()
    s1.close()


def merged(g, add, remove, num_atoms):
    rows = {int(a): (int(t), g["tgt_idx"][g["tgt_off"][r]:g["tgt_off"][r + 1]].tolist())
            for r, (a, t) in enumerate(zip(g["link_atom"], g["link_type"]))}
    for a in remove:
        rows.pop(int(a), None)
    rows.update(add)
    keys = sorted(rows)
    off = np.zeros(len(keys) + 1, np.int64)
    tg = []
    for r, k in enumerate(keys):
        tg += rows[k][1]
        off[r + 1] = len(tg)
    return dict(num_atoms=num_atoms, link_atom=np.array(keys, np.int32), tgt_off=off,
                tgt_idx=np.array(tg, np.int32), link_type=np.array([rows[k][0] for k in keys], np.int32))


@pytest.mark.parametrize("case", range(3))
def test_update_matches_rebuilt(case):
    """hgx_graph_update (atom added / removed events) == a snapshot built from the merged rows,
    including the lazily built type-grouped index and accumulators of the old rows."""
    from hypergraphdb_amd import HyperGraphSnapshot, _lib, pattern_batch
    rng = np.random.default_rng(80 + case)
    g = K.random_graph(rng, 250, 800, max_arity=6)
    snap = HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    pattern_batch(snap, random_queries(rng, g, 50))        # builds the type-grouped index
    check_batch(g, np.arange(32, dtype=np.int32), None, (True, True, False, False), snap=snap)
    # the multi-workgroup stage's per-seed bitmaps (sized by the old atom count) and the yield lists
    # of the old incidence must not survive the update
    snap.set_option(_lib.HGX_OPT_BFS_BLOCK, 2)
    check_batch(g, np.arange(16, dtype=np.int32), None, (False, True, False, False), lt=1, snap=snap)
    snap.set_option(_lib.HGX_OPT_BFS_BLOCK, 1)
    check_batch(g, np.arange(32, dtype=np.int32), None, (False, True, True, False), snap=snap)
    A0, grow = g["num_atoms"], [0, 40, 300][case]
    A1 = A0 + grow
    remove = rng.choice(g["link_atom"], 150, replace=False).tolist() + ([A0 + 5] if grow else [])  # + absent
    add = {}
    for a in range(A0, A1):
        if rng.random() < 0.6:
            k = int(rng.integers(0, 7))
            add[a] = (int(rng.integers(0, 3)), [int(x) for x in rng.integers(0, A1, k) if x != a])
    g2 = merged(g, add, remove, A1)
    snap.update(add=add, remove=remove, num_atoms=A1)
    assert snap.A == A1 and snap.M == len(g2["link_atom"])
    for k in ("link_atom", "tgt_off", "tgt_idx", "link_type"):
        np.testing.assert_array_equal(getattr(snap, k), g2[k], err_msg=k)
    check_all(snap, g2, rng)
    orc2 = oracle(g2)
    late = np.arange(max(0, A1 - 16), A1, dtype=np.int32)   # the appended atoms (the old bitmaps' tail)
    snap.set_option(_lib.HGX_OPT_BFS_BLOCK, 2)
    check_batch(g2, late, None, (False, True, False, False), lt=1, snap=snap, orc=orc2)
    check_batch(g2, late, None, (True, True, False, False), snap=snap, orc=orc2)
    snap.close()


def test_update_errors():
    from hypergraphdb_amd import HGXError, HyperGraphSnapshot, bfs_batch
    from hypergraphdb_amd import DefaultALGenerator
    g = K.random_graph(np.random.default_rng(90), 30, 40)
    snap = HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    la = int(g["link_atom"][0])
    with pytest.raises(HGXError, match="already exists"):
        snap.update(add={la: (0, [0])})
    with pytest.raises(HGXError, match="disappear"):
        snap.update(num_atoms=g["num_atoms"] - 1)
    with pytest.raises(HGXError):                             # target outside the rank space
        snap.update(add={g["num_atoms"]: (0, [g["num_atoms"] + 3])}, num_atoms=g["num_atoms"] + 1)
    res = bfs_batch(snap, [0, 1], 2, DefaultALGenerator(snap))
    with pytest.raises(HGXError, match="alive"):
        snap.update(remove=[la])
    res.close()
    snap.update(remove=[la])                                 # the graph is unchanged by the failures
    assert snap.M == len(g["link_atom"]) - 1
    snap.close()


def test_update_replace_rewrites_targets_and_type():
    """HyperGraph.replace keeps the handle and rewrites type + targets (C/HyperGraph.java:2100-2141,
    HGAtomReplacedEvent): the shim sends remove + add of the same link atom in one batch.  The new
    row takes the old rank slot; BFS, incidence and pattern results equal a rebuilt snapshot."""
    from hypergraphdb_amd import HyperGraphSnapshot
    rng = np.random.default_rng(95)
    g = K.random_graph(rng, 200, 600, max_arity=6)
    snap = HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    rep = [int(x) for x in rng.choice(g["link_atom"], 40, replace=False)]
    add = {a: (int(rng.integers(0, 3)), [int(x) for x in rng.integers(0, g["num_atoms"], int(rng.integers(0, 7)))
                                         if x != a]) for a in rep}
    g2 = merged(g, add, rep, g["num_atoms"])
    snap.update(add=add, remove=rep)
    assert snap.M == len(g["link_atom"])
    for k in ("link_atom", "tgt_off", "tgt_idx", "link_type"):
        np.testing.assert_array_equal(getattr(snap, k), g2[k], err_msg=k)
    check_all(snap, g2, rng)
    snap.close()


def test_sequence_refused_after_appended_ranks():
    """Appended ranks need not follow handle order, and the FIFO sequence cannot be repaired by a
    re-sort: hgx_bfs_sequence is refused until the caller re-asserts the order."""
    from hypergraphdb_amd import HGXError, HyperGraphSnapshot, bfs_sequence, _lib
    from test_gpu_seq import check_seq
    rng = np.random.default_rng(96)
    g = K.random_graph(rng, 120, 300, max_arity=5)
    snap = HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    A0 = g["num_atoms"]
    add = {A0 + 1: (0, [3, 7, 11]), A0 + 4: (1, [A0, 2])}
    snap.update(add=add, num_atoms=A0 + 6)
    with pytest.raises(HGXError, match="appended") as e:
        bfs_sequence(snap, [3], 3)
    assert e.value.code == _lib.HGX_E_UNSUPPORTED
    # IntHandleFactory handles are sequential: the appended ranks are in handle order -> re-assert
    snap.set_option(_lib.HGX_OPT_RANKS_ORDERED, 1)
    g2 = merged(g, add, [], A0 + 6)
    for mode in ((True, True, False, False), (False, True, False, False)):
        check_seq(g2, np.array([3, 7, A0], np.int32), None, mode, snap=snap)
    # an update that does not grow the rank space keeps the order
    snap.update(remove=[A0 + 1])
    assert bfs_sequence(snap, [3], 2).n_seeds == 1
    snap.close()
