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


def test_execution_contexts_run_side_by_side():
    """hgx_graph_context: contexts borrow the snapshot's arrays and run their own traversals; threads on
    different contexts get the serial results (default and ordered generator modes, pattern batches),
    a context keeps its snapshot alive after the snapshot handle is closed, and hgx_graph_update is
    refused while a context exists."""
    import hypergraphdb_amd as H
    from hypergraphdb_amd import AtomTypeCondition, DefaultALGenerator, synth
    from hypergraphdb_amd.query import pattern_batch_arrays
    g = synth.config5(scale=0.01, n_sources=256)
    snap = H.HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    T = g["subsumes_type"]
    gens = [DefaultALGenerator(snap, AtomTypeCondition(T), None, False, True, rev) for rev in (False, True)]
    seeds = g["seeds"]
    ref = []
    for gen in gens:
        r = H.bfs_batch(snap, seeds, None, gen)
        ref.append(r.counts())
        r.close()
    r = H.bfs_batch(snap, seeds, 3)
    ref.append(r.counts())
    r.close()
    orc = OracleGraph(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    from oracle_ctypes import algen
    oc, _ = orc.bfs_many(seeds[:16], -1, 4096, algen(T, False, True, True, False))
    assert np.array_equal(ref[1][:16], oc[:, :ref[1].shape[1]])

    ctxs = [snap.context() for _ in range(3)]
    ctx2 = ctxs[0].context()   # a context of a context is another context of the snapshot
    ctxs.append(ctx2)
    with pytest.raises(H.HGXError):
        snap.update(remove=[int(g["link_atom"][0])])
    errors, barrier = [], threading.Barrier(4)

    def worker(k):
        try:
            c = ctxs[k]
            gc = [DefaultALGenerator(c, AtomTypeCondition(T), None, False, True, rev) for rev in (False, True)]
            barrier.wait()
            for it in range(4):
                j = (k + it) % 3
                r = H.bfs_batch(c, seeds, 3) if j == 2 else H.bfs_batch(c, seeds, None, gc[j])
                got = r.counts()
                r.close()
                assert np.array_equal(got, ref[j]), (k, it, j)
        except Exception as e:   # noqa: BLE001 -- reported below
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th), "a worker hung"
    assert not errors, errors[:3]
    # the snapshot handle goes first; its contexts still traverse and query
    snap.close()
    r = H.bfs_batch(ctxs[1], seeds, None, DefaultALGenerator(ctxs[1], AtomTypeCondition(T), None, False, True, True))
    assert np.array_equal(r.counts(), ref[1])
    r.close()
    links = g["link_atom"][:50]
    q = pattern_batch_arrays(ctxs[2], np.full(50, -1, np.int32), np.arange(51, dtype=np.int64),
                             g["tgt_idx"][g["tgt_off"][:50]].astype(np.int32), np.zeros(50, np.int32),
                             np.zeros(51, np.int64), np.zeros(0, np.int32))
    for i in range(50):
        assert int(links[i]) in q[i].tolist()
    for c in ctxs:
        c.close()


def test_native_callers_coalesce():
    """20 native caller threads (tools/native/hgx_callers.cc, the JVM's threads in C: Python threads would
    serialise on the interpreter lock between calls) each issue single And queries on one graph, the
    usage of TC/query/QueryCompilation.java:76-122: every per-query hit count equals the oracle's, and
    with HGX_OPT_QUERY_COALESCE the engine serves them in fewer device batches than calls (off: one
    device batch per call)."""
    import ctypes as C
    import os

    import hypergraphdb_amd as H
    from hypergraphdb_amd import _lib, synth
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    L = C.CDLL(os.path.join(root, "tools", "native", "build", "libhgx_callers.so"))
    vp = C.c_void_p
    L.hgxc_pattern_threads.argtypes = [vp, C.c_int32, C.c_int32, vp, vp, vp, vp, vp, vp, C.c_int32, vp,
                                       C.POINTER(C.c_double)]
    g = synth.config3(scale=0.002, n_queries=3000)
    snap = H.HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    Q = g["queries"]
    nq = len(Q["type"])
    packed = [np.ascontiguousarray(Q["type"], np.int32), np.arange(nq + 1, dtype=np.int64),
              np.ascontiguousarray(Q["a"], np.int32), np.ones(nq, np.int32), np.arange(0, 3 * nq + 1, 3, dtype=np.int64),
              np.ascontiguousarray(np.stack([Q["x"], np.full(nq, -1, np.int32), Q["y"]], 1).reshape(-1), np.int32)]
    orc = OracleGraph(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    exp = np.array([len(orc.and_query(int(Q["type"][q]), [int(Q["a"][q])], (int(Q["x"][q]), -1, int(Q["y"][q]))))
                    for q in range(nq)], np.int64)
    for on in (1, 0):
        snap.set_option(_lib.HGX_OPT_QUERY_COALESCE, on)
        d0, c0, d1, c1 = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int64()
        _lib.lib().hgx_query_coalesce_stats(snap.handle, C.byref(d0), C.byref(c0))
        hits = np.zeros(nq, np.int64)
        sec = C.c_double()
        rc = L.hgxc_pattern_threads(snap.handle, 20, nq, *(a.ctypes.data for a in packed), 1, hits.ctypes.data,
                                    C.byref(sec))
        assert rc == 0, _lib.lib().hgx_last_error()
        assert np.array_equal(hits, exp), on
        _lib.lib().hgx_query_coalesce_stats(snap.handle, C.byref(d1), C.byref(c1))
        dev, calls = d1.value - d0.value, c1.value - c0.value
        if on:
            assert calls == nq and dev < calls // 2, (dev, calls)
        else:
            assert dev == calls == 0   # the direct path bypasses the combiner
    snap.close()
