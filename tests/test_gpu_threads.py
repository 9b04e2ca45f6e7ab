"""GPU: the threading contract of the boundary.  The reference runs one compiled
And from a 20-thread pool (testcore/test/java/hgtest/query/QueryCompilation.java:76-122); every
hgx_* entry point must be thread-safe.  20 host threads issue hgx_pattern_batch_packed and
hgx_bfs_batch on ONE graph at the same time; every result equals the serial one (and the oracle's).
ctypes releases the GIL around foreign calls, so the calls overlap inside libhgx."""
import threading

import numpy as np
import pytest

from oracle_ctypes import OracleGraph

pytestmark = pytest.mark.gpu


def test_twenty_threads_one_graph():
    import hypergraphdb_amd as H
    from hypergraphdb_amd import synth
    from hypergraphdb_amd.query import pattern_batch_arrays
    g = synth.config3(scale=0.002, n_queries=2000)
    snap = H.HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    Q = g["queries"]
    nq = len(Q["type"])
    packed = (Q["type"], np.arange(nq + 1, dtype=np.int64), Q["a"], np.ones(nq, np.int32),
              np.arange(0, 3 * nq + 1, 3, dtype=np.int64),
              np.stack([Q["x"], np.full(nq, -1, np.int32), Q["y"]], 1).reshape(-1))
    rng = np.random.default_rng(5)
    seed_sets = [rng.integers(0, g["n_nodes"], 64 + 32 * (k % 3)).astype(np.int32) for k in range(20)]
    # serial references
    ref_q = pattern_batch_arrays(snap, *packed)
    ref_b = []
    for seeds in seed_sets:
        r = H.bfs_batch(snap, seeds, 3)
        ref_b.append(r.counts())
        r.close()
    orc = OracleGraph(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    for k in (0, 7, 19):
        oc, _ = orc.bfs_many(seed_sets[k], 3, 4)
        n = ref_b[k].shape[1]
        assert n <= 4 and np.array_equal(ref_b[k], oc[:, :n]) and not oc[:, n:].any()
    for q in range(0, nq, 97):
        t, a, x, y = (int(Q[k][q]) for k in ("type", "a", "x", "y"))
        assert ref_q[q].tolist() == orc.and_query(t, [a], (x, -1, y)).tolist()

    errors, barrier = [], threading.Barrier(20)

    def worker(k):
        try:
            barrier.wait()
            for it in range(3):
                if (k + it) % 2 == 0:
                    r = pattern_batch_arrays(snap, *packed)
                    assert np.array_equal(r.offsets, ref_q.offsets) and np.array_equal(r.ids, ref_q.ids), (k, it)
                else:
                    r = H.bfs_batch(snap, seed_sets[k], 3)
                    c = r.counts()
                    r.close()
                    assert np.array_equal(c, ref_b[k]), (k, it)
        except Exception as e:   # noqa: BLE001 -- reported below
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(k,)) for k in range(20)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th), "a worker hung"
    assert not errors, errors[:3]
    snap.close()
