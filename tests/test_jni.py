"""The JNI shim executed on the CPU through a test JNIEnv (tests/jni_harness.py, tests/native/fake_jni.c).

No JDK exists in this image, so the shim's C is run the way a JVM would run it: the natives that need
no GPU (snapshot file, partition planner, shard tables, version / errors) against the Python mirror
of the same ABI, and every argument check the shim makes before the engine is called (inconsistent
lengths, offset tables that reach past their data array, null strings), plus OutOfMemory injection.
Every call also checks the JNI discipline the fake env records: pins released, inputs unmodified,
no JNI call with an exception pending.  The GPU natives run in tests/test_gpu_jni.py."""
import os

import numpy as np
import pytest

from jni_harness import JavaException, Jni, java_natives


@pytest.fixture
def jni():
    j = Jni()
    yield j
    j.close()


def small_graph(seed=3, N=300, M=500):
    from hypergraphdb_amd import synth
    g = synth.hypergraph(N, M, 2, 6, 2.1, 4, seed=seed)
    return g


def test_every_native_binds(jni):
    """Hgx.java's 67 declarations resolve to symbols of the shim with the declared arity."""
    nat = java_natives()
    assert len(nat) == 67
    for name in nat:
        jni._fn(name)


def test_version_error_devices(jni):
    assert jni.version().startswith("hgx ")
    assert isinstance(jni.lastError(), str)
    n = jni.deviceCount()
    assert n >= 0


def test_null_handles_throw_hgexception(jni):
    for name, args in (("graphInfo", (0,)), ("bfsInfo", (0,)), ("queryOffsets", (0,)), ("shardInfo", (0,)),
                       ("seqOffsets", (0,))):
        with pytest.raises(JavaException) as ei:
            jni.call(name, *args)
        assert ei.value.cls == "org.hypergraphdb.HGException", name


def test_snapshot_file_roundtrip(jni, tmp_path):
    from hypergraphdb_amd.snapshot import read_snapshot
    g = small_graph()
    A = g["num_atoms"]
    handles = (np.arange(A * 16) * 7 + 3).astype(np.int8)
    p = str(tmp_path / "s.hgcsr")
    jni.snapshotWrite(p, A, g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"], handles, 16)
    info = jni.snapshotInfo(p)
    assert info.tolist() == [A, len(g["link_atom"]), len(g["tgt_idx"]), 16, 1]
    hb = jni.snapshotHandles(p)
    assert np.array_equal(hb, handles)
    r = read_snapshot(p)
    for k in ("link_atom", "tgt_off", "tgt_idx", "link_type"):
        assert np.array_equal(r[k], g[k]), k
    # without handles: snapshotHandles returns null
    p2 = str(tmp_path / "s2.hgcsr")
    jni.snapshotWrite(p2, A, g["link_atom"], g["tgt_off"], g["tgt_idx"], None, None, 0)
    assert jni.snapshotHandles(p2) is None
    assert jni.snapshotInfo(p2).tolist()[3:] == [0, 0]
    with pytest.raises(JavaException) as ei:
        jni.snapshotInfo(str(tmp_path / "missing.hgcsr"))
    assert ei.value.cls == "org.hypergraphdb.HGException"


def test_snapshot_ranged_handles_and_streamed_writer(jni, tmp_path):
    """The readers / writer of handle tables beyond one Java array: snapshotHandlesRange returns any
    slice of the table (after one snapshotVerify), snapshotWriter* streams the table in pieces (odd
    piece sizes of 4-byte handles carry partial checksum words across calls) and writes a file
    byte-identical to snapshotWrite's; a short table, an abort or ranks outside the table are refused
    and leave no file behind."""
    g = small_graph()
    A = g["num_atoms"]
    rows = (g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    handles = ((np.arange(A * 4) * 13 + 5) % 251).astype(np.int8)
    ref = str(tmp_path / "ref.hgcsr")
    jni.snapshotWrite(ref, A, *rows, handles, 4)
    jni.snapshotVerify(ref)
    for first, n in ((0, A), (0, 1), (7, 100), (A - 3, 3), (A, 0)):
        assert np.array_equal(jni.snapshotHandlesRange(ref, first, n), handles[4 * first:4 * (first + n)])
    for first, n in ((A - 2, 3), (A + 1, 0), (-1, 2)):
        with pytest.raises(JavaException) as ei:
            jni.snapshotHandlesRange(ref, first, n)
        assert ei.value.cls == "java.lang.IllegalArgumentException"
    out = str(tmp_path / "streamed.hgcsr")
    w = jni.snapshotWriterBegin(out, A, *rows, 4)
    cuts = [0, 1, 4, 11, A // 2, A]
    for a, b in zip(cuts, cuts[1:]):
        jni.snapshotWriterHandles(w, handles[4 * a:4 * b].copy(), 4)
    jni.snapshotWriterEnd(w)
    assert open(out, "rb").read() == open(ref, "rb").read()
    jni.snapshotVerify(out)
    # a table one handle short: end refuses and removes the partial file
    bad = str(tmp_path / "short.hgcsr")
    w = jni.snapshotWriterBegin(bad, A, *rows, 4)
    jni.snapshotWriterHandles(w, handles[: 4 * (A - 1)].copy(), 4)
    with pytest.raises(JavaException):
        jni.snapshotWriterEnd(w)
    assert not os.path.exists(bad) and not os.path.exists(bad + ".tmp")
    w = jni.snapshotWriterBegin(bad, A, *rows, 4)
    with pytest.raises(JavaException):   # more handles than atoms
        jni.snapshotWriterHandles(w, np.zeros(4 * (A + 1), np.int8), 4)
    with pytest.raises(JavaException):   # not a whole number of handles
        jni.snapshotWriterHandles(w, np.zeros(6, np.int8), 4)
    jni.snapshotWriterAbort(w)
    assert not os.path.exists(bad) and not os.path.exists(bad + ".tmp")
    # a corrupted byte fails the verification but not the unverified ranged read
    data = bytearray(open(ref, "rb").read())
    data[-1] ^= 0x5A
    cor = str(tmp_path / "corrupt.hgcsr")
    open(cor, "wb").write(bytes(data))
    with pytest.raises(JavaException):
        jni.snapshotVerify(cor)
    assert len(jni.snapshotHandlesRange(cor, 0, 2)) == 8


def synthetic_header_file(path, A, hb):
    """A sparse .hgcsr of A atoms, no links and an all-zero handle table of A * hb bytes (header only
    written; the checksum field is left 0, so only unverified readers accept it)."""
    import struct
    hdr = struct.pack("<8sIIqqqIIQ8s", b"HGXCSR1\0", 2, 2, A, 0, 0, hb, 0, 0, b"\0" * 8)
    assert len(hdr) == 64
    tgt_off_at = 64                      # link_atom [0] at 64, tgt_off [1 x i64] at 64
    tbl_at = ((tgt_off_at + 8 + 63) // 64) * 64 + 0   # tgt_idx [0], link_type absent, then handles
    total = ((tbl_at + A * hb + 63) // 64) * 64
    with open(path, "wb") as f:
        f.write(hdr)
        f.truncate(total)                # sparse: no page of the table is ever written
    return tbl_at, total


def test_ranged_reader_of_a_300m_atom_table(jni, tmp_path):
    """A 300M-atom store with 16-byte UUID handles (4.8 GB of table, config 4's size): the whole-table
    reader throws cleanly (beyond one Java array), the ranged reader returns any slice of it."""
    A, hb = 300_000_000, 16
    p = str(tmp_path / "big.hgcsr")
    synthetic_header_file(p, A, hb)
    assert jni.snapshotInfo(p).tolist() == [A, 0, 0, hb, 0]
    with pytest.raises(JavaException) as ei:
        jni.snapshotHandles(p)
    assert ei.value.cls == "java.lang.UnsupportedOperationException"
    for first in (0, A // 2, A - 1000):
        page = jni.snapshotHandlesRange(p, first, 1000)
        assert len(page) == 1000 * hb and not page.any()
    with pytest.raises(JavaException) as ei:
        jni.snapshotHandlesRange(p, A - 10, 11)
    assert ei.value.cls == "java.lang.IllegalArgumentException"
    with pytest.raises(JavaException) as ei:   # 2^27 handles = 2 GiB: not one Java array
        jni.snapshotHandlesRange(p, 0, 1 << 27)
    assert ei.value.cls == "java.lang.UnsupportedOperationException"


def test_partition_natives_match_the_abi(jni):
    from hypergraphdb_amd.partition import Shard, partition_plan
    g = small_graph(seed=5, N=400, M=900)
    args = (g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    for NP in (1, 3, 4):
        plan = jni.partitionPlan(*args, NP)
        assert np.array_equal(plan, partition_plan(*args, NP))
        for part in range(NP):
            sh = jni.shardBuild(*args, NP, part, plan)
            try:
                ref = Shard.build(*args, NP, part, plan)
                assert jni.shardInfo(sh).tolist() == [ref.n_local, ref.n_owned, ref.n_links, ref.n_pins]
                assert np.array_equal(jni.shardLocalAtoms(sh), ref.export()["l2g"])
                assert np.array_equal(jni.shardOwners(sh), ref.exchange_tables()["xo_part"])
                ref.close()
            finally:
                jni.shardFree(sh)


BAD_ROWS = [
    ("tgtOff shorter than linkAtom + 1", lambda g: dict(tgt_off=g["tgt_off"][:-1])),
    ("tgtOff ends past tgtIdx", lambda g: dict(tgt_idx=g["tgt_idx"][:-3])),
    ("tgtOff does not start at 0", lambda g: dict(tgt_off=g["tgt_off"] + 1)),
    ("tgtOff decreases", lambda g: dict(tgt_off=np.concatenate([[0, 5, 3], g["tgt_off"][3:]]))),
    ("linkType length", lambda g: dict(link_type=g["link_type"][:-1])),
]


@pytest.mark.parametrize("what,mut", BAD_ROWS, ids=[b[0] for b in BAD_ROWS])
def test_shim_rejects_rows_that_would_read_past_java_arrays(jni, what, mut, tmp_path):
    """the ABI cannot know Java array lengths; the shim checks every offsets table against
    its data array and throws IllegalArgumentException before any engine call."""
    g = dict(small_graph())
    g.update(mut(g))
    rows = (g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    for name, args in (("graphCreate", rows + (0,)), ("partitionPlan", rows + (2,)),
                       ("shardBuild", rows + (2, 0, np.zeros(len(g["link_atom"]), np.int32))),
                       ("snapshotWrite", (str(tmp_path / "x.hgcsr"),) + rows + (None, 0))):
        with pytest.raises(JavaException) as ei:
            jni.call(name, *args)
        assert ei.value.cls == "java.lang.IllegalArgumentException", (name, ei.value)
    assert not os.path.exists(tmp_path / "x.hgcsr")


def test_shim_rejects_bad_pattern_batches(jni):
    n = 3
    ty = np.zeros(n, np.int32)
    ok = dict(incOff=np.array([0, 1, 2, 3]), inc=np.array([1, 2, 3]), hasOrdered=np.zeros(n, np.int32),
              patOff=np.zeros(n + 1, np.int64), pat=np.zeros(0, np.int32))
    cases = [dict(incOff=np.array([0, 1, 2, 4])),            # ends past inc
             dict(incOff=np.array([0, 2, 1, 3])),            # decreases
             dict(incOff=np.array([1, 1, 2, 3])),            # does not start at 0
             dict(hasOrdered=np.zeros(n + 1, np.int32)),     # length
             dict(patOff=np.array([0, 0, 0, 1]))]            # ends past pat
    for c in cases:
        a = dict(ok, **c)
        for name in ("patternBatch", "patternBatchStructs"):
            with pytest.raises(JavaException) as ei:
                jni.call(name, 1, ty, a["incOff"], a["inc"], a["hasOrdered"], a["patOff"], a["pat"])
            assert ei.value.cls == "java.lang.IllegalArgumentException", (name, c)
    # the ext form: a positioned record is 4 ints; pattern sets index patOff
    z = np.zeros(n + 1, np.int64)
    base = dict(typeOff=z, types=np.zeros(0, np.int32), incOff=np.array([0, 1, 2, 3]), inc=np.array([1, 2, 3]),
                posOff=z, pos=np.zeros(0, np.int32), psetOff=z, patOff=np.zeros(1, np.int64),
                pat=np.zeros(0, np.int32), arity=np.full(n, -1, np.int32))
    bad = [dict(posOff=np.array([0, 0, 0, 1]), pos=np.zeros(3, np.int32)),   # one record needs 4 ints
           dict(psetOff=np.array([0, 0, 0, 1])),                              # a set with no patOff entry
           dict(psetOff=np.array([0, 0, 0, 1]), patOff=np.array([0, 2]), pat=np.zeros(1, np.int32)),
           dict(typeOff=np.array([0, 0, 0, 1]))]
    for c in bad:
        a = dict(base, **c)
        with pytest.raises(JavaException) as ei:
            jni.patternBatchExt(1, a["typeOff"], a["types"], a["incOff"], a["inc"], a["posOff"], a["pos"],
                                a["psetOff"], a["patOff"], a["pat"], a["arity"])
        assert ei.value.cls == "java.lang.IllegalArgumentException", c


def test_null_strings_and_rccl_id(jni):
    with pytest.raises(JavaException) as ei:
        jni.graphOpen(None, 0)
    assert ei.value.cls == "java.lang.NullPointerException"
    with pytest.raises(JavaException) as ei:
        jni.rcclCreate(np.zeros(5, np.int8), 1, 0, 0)
    assert ei.value.cls == "java.lang.IllegalArgumentException"


def test_out_of_memory_injection_releases_everything(jni, tmp_path):
    """A VM may fail any pin or allocation with OutOfMemoryError: the shim returns at once, releases
    what it pinned and makes no further JNI call with the exception pending."""
    g = small_graph()
    rows = (g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    for nth in range(1, 6):
        jni.inject_oom(nth)
        with pytest.raises(JavaException) as ei:
            jni.partitionPlan(*rows, 2)
        assert ei.value.cls == "java.lang.OutOfMemoryError", nth
    jni.inject_oom(0)
    assert len(jni.partitionPlan(*rows, 2)) == len(g["link_atom"])


def test_graph_create_without_a_gpu_throws(jni):
    if jni.deviceCount() > 0:
        pytest.skip("a GPU is visible: covered by tests/test_gpu_jni.py")
    g = small_graph()
    with pytest.raises(JavaException) as ei:
        jni.graphCreate(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"], 0)
    assert ei.value.cls == "org.hypergraphdb.HGException"
