"""CPU tests of the boundary: libhgx.so loads and exports every symbol include/hgx.h declares;
host-side logic (handle ranking, And normalisation, generator determinism).  No GPU compute."""
import ctypes as C
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "hgx.h")).read()
    return sorted(set(re.findall(r"\b(hgx_[a-z_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    from hypergraphdb_amd import _lib
    L = C.CDLL(_lib.LIB_PATH)
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(L, s), s
    assert sorted(_lib.EXPORTED) == syms


def test_exports_are_c_abi():
    """extern "C": the exported names are unmangled."""
    out = os.popen(f"nm -D --defined-only {os.path.join(ROOT, 'hypergraphdb_amd', 'libhgx.so')}").read()
    for s in header_symbols():
        assert re.search(rf"\sT {s}$", out, re.M), s


def test_version_and_error_without_gpu():
    from hypergraphdb_amd import _lib
    L = _lib.lib()
    assert L.hgx_version().decode().startswith("hgx ")
    # a null descriptor is rejected with a status, never a crash
    h = C.c_void_p()
    assert L.hgx_graph_create(None, 0, C.byref(h)) == _lib.HGX_E_INVALID
    assert b"null" in L.hgx_last_error()


def test_handle_ranking_is_byte_order():
    """IntPersistentHandle bytes = x ^ 0x80000000 big-endian (BAUtils.java:69-80): rank == int order;
    UUID handles: unsigned lexicographic (UUID.java:364-376)."""
    from hypergraphdb_amd.snapshot import handle_bytes, rank_handles
    ints = [1000, -5, 7, 2**31 - 1, -2**31, 0]
    r = rank_handles(ints)
    assert [h for h, _ in sorted(r.items(), key=lambda kv: kv[1])] == sorted(ints)
    assert handle_bytes(1000) == bytes([0x80, 0x00, 0x03, 0xE8])
    uu = [bytes([0xFF] + [0] * 15), bytes([0x01] + [0] * 15), bytes([0x7F] + [9] * 15)]
    r = rank_handles(uu)
    assert r[uu[1]] == 0 and r[uu[2]] == 1 and r[uu[0]] == 2


def test_and_normalisation():
    from hypergraphdb_amd import HGXUnsupported, hg
    from hypergraphdb_amd.query import normalize
    q = normalize(hg.and_(hg.type(3), hg.incident(5), hg.and_(hg.orderedLink(1, hg.anyHandle(), 2))))
    assert q == {"types": [3], "inc": [5], "pos": [], "patterns": [(1, -1, 2)], "arity": -1}
    # several orderedLinks are predicates of one And; LinkCondition expands to incidents (ANY dropped)
    q = normalize(hg.and_(hg.orderedLink(1), hg.orderedLink(2), hg.link(7, hg.anyHandle(), 8)))
    assert q["patterns"] == [(1,), (2,)] and q["inc"] == [7, 8]
    q = normalize(hg.and_(hg.incidentAt(4, -1), hg.incidentNotAt(5, 0, 2), hg.arity(3), hg.typePlus([2, 1])))
    assert q["pos"] == [(4, -1, -1, 0), (5, 0, 2, 1)] and q["arity"] == 3 and q["types"] == [1, 2]
    # every type condition must hold: typePlus sets intersect with exact types
    assert normalize(hg.and_(hg.typePlus([1, 2]), hg.type(2), hg.incident(0)))["types"] == [2]
    assert normalize(hg.and_(hg.type(1), hg.type(2), hg.incident(0))) == "empty"
    assert normalize(hg.and_(hg.arity(1), hg.arity(2), hg.incident(0))) == "empty"
    with pytest.raises(HGXUnsupported):
        normalize(hg.and_(hg.incident(1), hg.bfs(2)))


def test_generator_deterministic_and_valid():
    from hypergraphdb_amd import synth
    a = synth.hypergraph(1000, 3000, 2, 8, 2.1, 4, seed=42)
    b = synth.hypergraph(1000, 3000, 2, 8, 2.1, 4, seed=42)
    for k in ("tgt_off", "tgt_idx", "link_type"):
        assert np.array_equal(a[k], b[k])
    off, tg = a["tgt_off"], a["tgt_idx"]
    assert tg.min() >= 0 and tg.max() < 1000
    ar = np.diff(off)
    assert ar.min() >= 2 and ar.max() <= 8
    for r in range(0, 3000, 97):   # distinct targets within a link
        row = tg[off[r]:off[r + 1]]
        assert len(set(row.tolist())) == len(row)
    # power law: node 0 is the heaviest
    deg = np.bincount(tg, minlength=1000)
    assert deg[0] == deg.max()


def test_generator_ontology_shape():
    from hypergraphdb_amd import synth
    g = synth.config5(scale=1e-3)
    tg = g["tgt_idx"].reshape(-1, 2)
    sub = g["link_type"] == g["subsumes_type"]
    assert (tg[sub, 0] < tg[sub, 1]).all()          # parents have lower ids (a DAG)
    assert (tg[:, 0] != tg[:, 1]).all()


JAVA = os.path.join(ROOT, "java")


def test_jni_shim_compiles():
    """java/jni/hgx_jni.c type-checks against include/hgx.h (a minimal jni.h stands in for the JDK's:
    no JDK in this image).  Catches ABI drift between the C ABI and the JNI shim."""
    import shutil
    import subprocess
    gcc = shutil.which("gcc")
    assert gcc
    r = subprocess.run([gcc, "-std=c99", "-Wall", "-Werror", "-fsyntax-only", "-I", os.path.join(ROOT, "tests", "jni_stub"),
                        "-I", os.path.join(ROOT, "include"), os.path.join(JAVA, "jni", "hgx_jni.c")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_every_java_native_has_a_body_and_every_abi_entry_a_java_caller():
    """Hgx.java's natives <-> hgx_jni.c's JNI functions, and every hgx_* entry point of include/hgx.h
    is called by the shim (hgx_comm_host_create excepted: its collectives are host callbacks, and
    the JNI contract has no callbacks into the JVM; and the transport diagnostic
    hgx_comm_check_allgather, which only the tests call)."""
    import re
    java = open(os.path.join(JAVA, "org", "hypergraphdb", "gpu", "Hgx.java")).read()
    jni = open(os.path.join(JAVA, "jni", "hgx_jni.c")).read()
    natives = set(re.findall(r"static native [\w\[\]<>]+ (\w+)\(", java))
    bodies = set(re.findall(r"JNIEXPORT [\w ]+ JFN\((\w+)\)", jni))
    assert natives == bodies, (sorted(natives - bodies), sorted(bodies - natives))
    header = open(os.path.join(ROOT, "include", "hgx.h")).read()
    entries = set(re.findall(r"^\s*(?:int|void|const char \*)\s+\*?(hgx_\w+)\(", header, re.M))
    called = set(re.findall(r"\b(hgx_\w+)\(", jni))
    missing = sorted(entries - called - {"hgx_comm_host_create", "hgx_comm_check_allgather"})
    assert not missing, missing
