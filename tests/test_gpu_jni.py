"""GPU parity through the JNI shim: every native of Hgx.java executed against the oracle.

No JDK exists in this image, so the shim (java/jni/hgx_jni.c) runs under a
test JNIEnv (tests/native/fake_jni.c via tests/jni_harness.py) that models Java arrays, copy-mode
pinning and pending exceptions, and checks the JNI discipline on every call.  This is the path
HGGpuSnapshot / HGGpuTraversal / GpuAndToQuery / GpuTraversalToQuery take (java/org/hypergraphdb/gpu):
the results are compared with the C oracle (oracle/hgx_oracle.c, the restatement of
HGBreadthFirstTraversal / DefaultALGenerator / AndToQuery), bit-exact.  The last test checks that
all 67 natives were called."""
import numpy as np
import pytest

import kat_graphs as K
from jni_harness import JavaException, Jni, java_natives
from oracle_ctypes import OracleGraph, algen

pytestmark = pytest.mark.gpu

MODES = K.ALGEN_MODES


@pytest.fixture(scope="module")
def jni():
    j = Jni()
    yield j
    j.close()


@pytest.fixture(scope="module")
def graph():
    rng = np.random.default_rng(4242)
    g = K.random_graph(rng, 700, 1600, max_arity=7, link_targets=True, n_types=3)
    orc = OracleGraph(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    return g, orc


def rows(g):
    return (g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])


@pytest.fixture(scope="module")
def gh(jni, graph):
    g, _ = graph
    h = jni.graphCreate(*rows(g), 0)
    assert h != 0
    yield h
    jni.graphDestroy(h)


def test_device(jni):
    assert jni.deviceCount() >= 1
    jni.deviceSynchronize(0)
    assert jni.version().startswith("hgx ")


def test_graph_info_incidence_degree_export(jni, graph, gh):
    g, orc = graph
    A, M, I = jni.graphInfo(gh).tolist()
    atoms = np.arange(g["num_atoms"], dtype=np.int32)
    inc = [orc.incidence(int(a)) for a in atoms]
    assert (A, M, I) == (g["num_atoms"], len(g["link_atom"]), sum(len(x) for x in inc))
    assert np.array_equal(jni.degree(gh, atoms), np.array([len(x) for x in inc], np.int64))
    for a in range(0, g["num_atoms"], 7):
        assert np.array_equal(jni.incidence(gh, a), inc[a]), a
    assert np.array_equal(jni.graphExportLinks(gh), g["link_atom"])
    assert np.array_equal(jni.graphExportOffsets(gh), g["tgt_off"])
    assert np.array_equal(jni.graphExportTargets(gh), g["tgt_idx"])
    with pytest.raises(JavaException) as ei:
        jni.incidence(gh, g["num_atoms"] + 5)
    assert ei.value.cls == "org.hypergraphdb.HGException"


@pytest.mark.parametrize("mi", range(len(MODES)))
def test_bfs_batch_every_mode_vs_oracle(jni, graph, gh, mi):
    """bfsBatch + bfsInfo / bfsCounts / bfsVisited / bfsDepthOf / bfsStats / bfsFree: what
    HGGpuTraversal.bfsBatch and GpuTraversalToQuery run."""
    g, orc = graph
    P, S, R, RS = MODES[mi]
    lt = -1 if mi % 3 else int(mi % 2)
    seeds = np.random.default_rng(mi).integers(0, g["num_atoms"], 70).astype(np.int32)
    maxd = [-1, 2, 3][mi % 3]
    jni.setTiming(gh, True)
    r = jni.bfsBatch(gh, seeds, maxd, lt, P, S, R, RS)
    try:
        ns, nl = jni.bfsInfo(r).tolist()
        assert ns == len(seeds)
        counts = jni.bfsCounts(r).reshape(ns, nl)
        trav = 0
        for i, s in enumerate(seeds):
            lv = orc.bfs_levels(int(s), maxd, algen(lt, P, S, R, RS))
            _, _, _, tr = orc.bfs(int(s), maxd, algen(lt, P, S, R, RS))
            trav += tr
            for d in range(nl):
                exp = lv[d] if d < len(lv) else np.zeros(0, np.int32)
                assert counts[i, d] == len(exp), (i, d)
                if i % 9 == 0:
                    assert np.array_equal(jni.bfsVisited(r, i, d), exp), (i, d)
                    # paged reads (bfsVisitedRange): pages of 3 reassemble the set
                    pages = [jni.bfsVisitedRange(r, i, d, f, 3) for f in range(0, len(exp) + 3, 3)]
                    assert np.array_equal(np.concatenate(pages), exp), (i, d)
            if i % 9 == 0:
                for d, lvl in enumerate(lv):
                    for a in lvl[:3]:
                        assert jni.bfsDepthOf(r, i, int(a)) == d
        st = jni.bfsStats(r, True)
        assert st[1] == float(trav)      # the hyperedge-TEPS numerator equals the oracle's
        assert st[0] >= 0.0
    finally:
        jni.bfsFree(r)
    jni.setTiming(gh, False)


def test_graph_context(jni, graph, gh):
    """graphContext: an execution context of the snapshot (one per concurrent Java caller) traverses
    like the snapshot itself and outlives nothing it borrows (destroyed first here)."""
    g, orc = graph
    c = jni.graphContext(gh)
    assert c != 0 and c != gh
    try:
        assert jni.graphInfo(c).tolist() == jni.graphInfo(gh).tolist()
        seeds = np.arange(0, 60, dtype=np.int32)
        r = jni.bfsBatch(c, seeds, 2, -1, True, True, False, False)
        try:
            ns, nl = jni.bfsInfo(r).tolist()
            counts = jni.bfsCounts(r).reshape(ns, nl)
            for i in range(0, 60, 7):
                lv = orc.bfs_levels(int(seeds[i]), 2)
                assert counts[i, :len(lv)].tolist() == [len(x) for x in lv]
        finally:
            jni.bfsFree(r)
    finally:
        jni.graphDestroy(c)


def test_bfs_sequence_order_exact(jni, graph, gh):
    """bfsSequence + seqOffsets / seqLinks / seqAtoms / seqDists / seqStats / seqFree: the
    HGGpuTraversal.next() sequence, FIFO order and discovering links included."""
    g, orc = graph
    for mi in (0, 3, 5):
        P, S, R, RS = MODES[mi]
        seeds = np.random.default_rng(100 + mi).integers(0, g["num_atoms"], 12).astype(np.int32)
        s = jni.bfsSequence(gh, seeds, -1, -1, P, S, R, RS)
        try:
            off = jni.seqOffsets(s)
            links, atoms, dists = jni.seqLinks(s), jni.seqAtoms(s), jni.seqDists(s)
            trav = 0
            for i, sd in enumerate(seeds):
                l, a, d, tr = orc.bfs(int(sd), -1, algen(-1, P, S, R, RS))
                trav += tr
                sl = slice(int(off[i]), int(off[i + 1]))
                assert np.array_equal(atoms[sl], a) and np.array_equal(links[sl], l) and np.array_equal(dists[sl], d)
            assert jni.seqStats(s)[1] == float(trav)
            # paged column reads (seqRange) across seed boundaries, and the engine split
            for which, col in ((0, links), (1, atoms), (2, dists)):
                got = np.concatenate([jni.seqRange(s, which, f, 5) for f in range(0, len(col) + 5, 5)])
                assert np.array_equal(got, col), which
            nb, nl, _pull, _grid = jni.seqEngineStats(s).tolist()
            assert nb + nl == len(seeds)
        finally:
            jni.seqFree(s)


def pattern_queries(g, rng, n):
    """And{type, incident(a), orderedLink(x, ANY, y)} from sampled links (+ negatives)."""
    off, tg, lt = g["tgt_off"], g["tgt_idx"], g["link_type"]
    qs = []
    while len(qs) < n:
        r = int(rng.integers(0, len(g["link_atom"])))
        t = tg[off[r]:off[r + 1]]
        if len(t) < 3:
            continue
        a = int(t[int(rng.integers(0, len(t)))]) if rng.random() < 0.8 else int(rng.integers(0, g["num_atoms"]))
        qs.append((int(lt[r]) if rng.random() < 0.8 else -1, [a], (int(t[0]), -1, int(t[2])) if rng.random() < 0.7 else None))
    return qs


def packed(qs):
    n = len(qs)
    ty = np.array([q[0] for q in qs], np.int32)
    io = np.zeros(n + 1, np.int64)
    po = np.zeros(n + 1, np.int64)
    inc, pat, ho = [], [], np.zeros(n, np.int32)
    for i, (t, a, p) in enumerate(qs):
        inc += a
        io[i + 1] = len(inc)
        if p is not None:
            ho[i] = 1
            pat += list(p)
        po[i + 1] = len(pat)
    return ty, io, np.array(inc, np.int32), ho, po, np.array(pat, np.int32)


def test_pattern_batches_vs_oracle(jni, graph, gh):
    """patternBatch / patternBatchStructs + queryOffsets / queryIds / queryMs / queryFree: the
    GpuAndToQuery batch path."""
    g, orc = graph
    qs = pattern_queries(g, np.random.default_rng(7), 300)
    args = packed(qs)
    exp = [orc.and_query(t, a, p) for t, a, p in qs]
    jni.setTiming(gh, True)
    for fn in ("patternBatch", "patternBatchStructs"):
        q = jni.call(fn, gh, *args)
        try:
            off, ids = jni.queryOffsets(q), jni.queryIds(q)
            assert len(off) == len(qs) + 1
            for i, e in enumerate(exp):
                assert np.array_equal(ids[off[i]:off[i + 1]], e), (fn, i, qs[i])
            ms = jni.queryMs(q)
            assert len(ms) == 3 and ms[0] >= 0
        finally:
            jni.queryFree(q)
    jni.setTiming(gh, False)
    # a resident query set (querySetCreate / patternBatchSet / querySetFree), run twice
    qset = jni.querySetCreate(gh, *args)
    try:
        for _ in range(2):
            q = jni.patternBatchSet(gh, qset)
            try:
                off, ids = jni.queryOffsets(q), jni.queryIds(q)
                for i, e in enumerate(exp):
                    assert np.array_equal(ids[off[i]:off[i + 1]], e), ("set", i)
            finally:
                jni.queryFree(q)
        # into caller arrays (patternBatchSetInto): exact fit, then an ids array one short
        total = sum(len(e) for e in exp)
        off = np.zeros(len(exp) + 1, np.int64)
        ids = np.full(total, -1, np.int32)
        assert jni.patternBatchSetInto(gh, qset, off, ids) == total
        for i, e in enumerate(exp):
            assert np.array_equal(ids[off[i]:off[i + 1]], e), ("set into", i)
        short = np.full(max(total - 1, 0), -1, np.int32)
        off[:] = 0
        assert jni.patternBatchSetInto(gh, qset, off, short) == total
        assert off[-1] == total and (short == -1).all()
        with pytest.raises(JavaException):
            jni.patternBatchSetInto(gh, qset, None, ids)
        # an offsets array shorter than the set's n + 1 is refused before the engine writes into it
        # (the engine always writes n + 1 offsets)
        guard = np.full(len(exp) + 8, -7, np.int64)
        with pytest.raises(JavaException) as ei:
            jni.patternBatchSetInto(gh, qset, guard[: len(exp)], ids)
        assert ei.value.cls == "java.lang.IllegalArgumentException"
        assert (guard == -7).all()
    finally:
        jni.querySetFree(qset)
    # no incidence anchor: the engine refuses, the Java side keeps AndToQuery
    with pytest.raises(JavaException) as ei:
        jni.patternBatch(gh, np.array([1], np.int32), np.zeros(2, np.int64), np.zeros(0, np.int32),
                         np.zeros(1, np.int32), np.zeros(2, np.int64), np.zeros(0, np.int32))
    assert ei.value.cls == "java.lang.UnsupportedOperationException"


def test_pattern_batch_ext_vs_oracle(jni, graph, gh):
    """patternBatchExt: TypePlus (several types), positioned incidents, several orderedLinks, arity."""
    g, orc = graph
    rng = np.random.default_rng(11)
    off, tg = g["tgt_off"], g["tgt_idx"]
    qs = []
    while len(qs) < 120:
        r = int(rng.integers(0, len(g["link_atom"])))
        t = tg[off[r]:off[r + 1]]
        if len(t) < 2:
            continue
        types = [] if rng.random() < 0.3 else sorted({int(g["link_type"][r]), int(rng.integers(0, 3))})
        inc = [int(t[-1])] if rng.random() < 0.5 else []
        pos = [(int(t[0]), 0, int(rng.integers(0, 3)), int(rng.random() < 0.2))]
        pats = [(int(t[0]), -1)] if rng.random() < 0.5 else [(int(t[0]),), (int(t[-1]),)]
        ar = int(len(t)) if rng.random() < 0.3 else -1
        qs.append((types, inc, pos, pats, ar))
    n = len(qs)
    to, io, po, so = (np.zeros(n + 1, np.int64) for _ in range(4))
    types, inc, pos, patoff, pat, ar = [], [], [], [0], [], np.zeros(n, np.int32)
    for i, (ty, ic, ps, pts, a) in enumerate(qs):
        types += ty
        to[i + 1] = len(types)
        inc += ic
        io[i + 1] = len(inc)
        for p in ps:
            pos += list(p)
        po[i + 1] = len(pos) // 4
        for p in pts:
            pat += list(p)
            patoff.append(len(pat))
        so[i + 1] = len(patoff) - 1
        ar[i] = a
    q = jni.patternBatchExt(gh, to, np.array(types, np.int32), io, np.array(inc, np.int32), po,
                            np.array(pos, np.int32), so, np.array(patoff, np.int64), np.array(pat, np.int32), ar)
    try:
        off_, ids = jni.queryOffsets(q), jni.queryIds(q)
        for i, (ty, ic, ps, pts, a) in enumerate(qs):
            e = orc.and_query_ext(ty, ic, ps, pts, a)
            assert np.array_equal(ids[off_[i]:off_[i + 1]], e), (i, qs[i])
    finally:
        jni.queryFree(q)


def test_snapshot_file_open_update(jni, graph, tmp_path):
    """snapshotWrite / snapshotInfo / snapshotHandles / graphOpen / graphUpdate / setOption: the
    HGGpuSnapshot export, reopen and event-batch path, against the oracle on the updated rows."""
    g, orc = graph
    A = g["num_atoms"]
    handles = (np.arange(A * 4) % 251).astype(np.int8)
    p = str(tmp_path / "g.hgcsr")
    jni.snapshotWrite(p, *rows(g), handles, 4)
    assert jni.snapshotInfo(p).tolist() == [A, len(g["link_atom"]), len(g["tgt_idx"]), 4, 1]
    assert np.array_equal(jni.snapshotHandles(p), handles)
    # the streamed writer (the exporter of tables beyond one byte[]) and the ranged reader
    p2 = str(tmp_path / "g2.hgcsr")
    w = jni.snapshotWriterBegin(p2, *rows(g), 4)
    jni.snapshotWriterHandles(w, handles[:4 * 5].copy(), 4)
    jni.snapshotWriterHandles(w, handles[4 * 5:].copy(), 4)
    jni.snapshotWriterEnd(w)
    assert open(p2, "rb").read() == open(p, "rb").read()
    jni.snapshotVerify(p2)
    assert np.array_equal(jni.snapshotHandlesRange(p2, 3, 9), handles[12:48])
    w = jni.snapshotWriterBegin(str(tmp_path / "g3.hgcsr"), *rows(g), 4)
    jni.snapshotWriterAbort(w)
    h = jni.graphOpen(p, 0)
    try:
        assert jni.graphInfo(h).tolist()[:2] == [A, len(g["link_atom"])]
        # remove two links, add one new link atom (a new rank) targeting existing atoms
        rm = g["link_atom"][[3, 10]].astype(np.int32)
        new_atom = A
        add_t = np.array([int(g["tgt_idx"][0]), int(g["tgt_idx"][5]), 1], np.int32)
        jni.graphUpdate(h, A + 1, np.array([new_atom], np.int32), np.array([0, 3], np.int64), add_t,
                        np.array([2], np.int32), rm)
        keep = np.ones(len(g["link_atom"]), bool)
        keep[[3, 10]] = False
        off = g["tgt_off"]
        la2, tg2, off2, ty2 = [], [], [0], []
        for r in np.nonzero(keep)[0]:
            la2.append(int(g["link_atom"][r]))
            tg2 += g["tgt_idx"][off[r]:off[r + 1]].tolist()
            off2.append(len(tg2))
            ty2.append(int(g["link_type"][r]))
        la2.append(new_atom)
        tg2 += add_t.tolist()
        off2.append(len(tg2))
        ty2.append(2)
        o2 = OracleGraph(A + 1, np.array(la2, np.int32), np.array(off2, np.int64), np.array(tg2, np.int32),
                         np.array(ty2, np.int32))
        assert np.array_equal(jni.graphExportLinks(h), np.array(la2, np.int32))
        for a in list(range(0, A, 11)) + [int(add_t[0]), 1]:
            assert np.array_equal(jni.incidence(h, a), o2.incidence(a)), a
        # an update appended a rank: the order-exact traversal refuses until the caller re-asserts it
        with pytest.raises(JavaException) as ei:
            jni.bfsSequence(h, np.array([1], np.int32), 2, -1, True, True, False, False)
        assert ei.value.cls == "java.lang.UnsupportedOperationException"
        jni.setOption(h, 3, 1)   # HGX_OPT_RANKS_ORDERED: the new handle sorts after every old one
        s = jni.bfsSequence(h, np.array([1], np.int32), 2, -1, True, True, False, False)
        try:
            l, a, d, _ = o2.bfs(1, 2, algen())
            assert np.array_equal(jni.seqAtoms(s), a) and np.array_equal(jni.seqLinks(s), l)
        finally:
            jni.seqFree(s)
    finally:
        jni.graphDestroy(h)


def test_partitioned_natives_vs_oracle(jni, graph):
    """partitionPlan / shardBuild / shardInfo / shardLocalAtoms / shardOwners / shardGraphCreate /
    pbfsBatchGroup / shardFree, and the RCCL path at world 1: rcclUniqueId / rcclCreate / pbfsBatch /
    commDestroy (config 4's per-JVM shape)."""
    g, orc = graph
    seeds = np.random.default_rng(5).integers(0, g["num_atoms"], 40).astype(np.int32)
    exp = [orc.bfs_levels(int(s), 3) for s in seeds]
    NP = 3
    plan = jni.partitionPlan(*rows(g), NP)
    shards, graphs = [], []
    try:
        for p in range(NP):
            sh = jni.shardBuild(*rows(g), NP, p, plan)
            shards.append(sh)
            info = jni.shardInfo(sh)
            l2g = jni.shardLocalAtoms(sh)
            own = jni.shardOwners(sh)
            assert len(l2g) == info[0] == len(own) and int((own < 0).sum()) == info[1]
            graphs.append(jni.shardGraphCreate(sh, 0))
        res = jni.pbfsBatchGroup(np.array(graphs, np.int64), seeds, 3, -1, True, True, False, False)
        try:
            total = None
            for r in res:
                c = jni.bfsCounts(r).reshape(len(seeds), -1)
                total = c if total is None else total + c
            for i, lv in enumerate(exp):
                assert total[i, :len(lv)].tolist() == [len(x) for x in lv], i
                if i % 8 == 0:
                    for d, lvl in enumerate(lv):
                        got = np.sort(np.concatenate([jni.bfsVisited(r, i, d) for r in res]))
                        assert np.array_equal(got, lvl), (i, d)
        finally:
            for r in res:
                jni.bfsFree(int(r))
    finally:
        for x in graphs:
            jni.graphDestroy(x)
        for sh in shards:
            jni.shardFree(sh)
    # one part over RCCL at world 1 (the driver's multi-GPU bench runs world > 1)
    plan1 = jni.partitionPlan(*rows(g), 1)
    sh = jni.shardBuild(*rows(g), 1, 0, plan1)
    gp = jni.shardGraphCreate(sh, 0)
    jni.shardFree(sh)
    uid = jni.rcclUniqueId()
    assert len(uid) == 128
    comm = jni.rcclCreate(uid, 1, 0, 0)
    try:
        r = jni.pbfsBatch(gp, comm, seeds, 3, -1, True, True, False, False)
        try:
            c = jni.bfsCounts(r).reshape(len(seeds), -1)
            for i, lv in enumerate(exp):
                assert c[i, :len(lv)].tolist() == [len(x) for x in lv], i
            assert jni.bfsStats(r, False)[0] >= 0.0
        finally:
            jni.bfsFree(r)
    finally:
        jni.commDestroy(comm)
        jni.graphDestroy(gp)


def test_concurrent_single_queries_coalesce(jni, graph, gh):
    """20 'Java threads' (one JNIEnv each) issue single And queries at once, the usage of
    TC/query/QueryCompilation.java:76-122: every result equals the oracle's and queryCoalesceStats counts
    every call (HGX_OPT_QUERY_COALESCE)."""
    import threading
    g, orc = graph
    qs = pattern_queries(g, np.random.default_rng(21), 400)
    exp = [orc.and_query(t, a, p) for t, a, p in qs]
    b0 = jni.queryCoalesceStats(gh)
    errors = []

    def worker(t):
        j = Jni()
        try:
            for i in range(t, len(qs), 20):
                q = j.patternBatch(gh, *packed([qs[i]]))
                try:
                    ids = j.queryIds(q)
                    if not np.array_equal(ids, exp[i]):
                        errors.append((t, i))
                finally:
                    j.queryFree(q)
        except Exception as e:   # noqa: BLE001 - reported below
            errors.append((t, repr(e)))
        finally:
            j.close()

    th = [threading.Thread(target=worker, args=(t,)) for t in range(20)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors[:5]
    b1 = jni.queryCoalesceStats(gh)
    dev, calls = int(b1[0] - b0[0]), int(b1[1] - b0[1])
    assert calls == len(qs)
    # Python 'Java threads' hold the interpreter lock between calls, so whether two single queries are in
    # the engine at once is up to the interpreter's scheduling; the coalescing factor itself is asserted
    # with native caller threads (tests/test_gpu_threads.py::test_native_callers_coalesce).
    assert 1 <= dev <= calls, (dev, calls)


def test_engine_errors_become_exceptions(jni, gh):
    with pytest.raises(JavaException) as ei:
        jni.bfsBatch(gh, np.array([10 ** 8], np.int32), 2, -1, True, True, False, False)
    assert ei.value.cls == "org.hypergraphdb.HGException"
    assert "seed" in ei.value.msg or "range" in ei.value.msg
    assert jni.lastError() == ei.value.msg


def test_all_natives_were_executed(jni):
    """Runs last (file order): every native declared in Hgx.java has been called on the GPU."""
    missing = sorted(set(java_natives()) - jni.called)
    assert not missing, missing
    assert len(jni.called) == 67
