"""CPU tests of the snapshot on disk (.hgcsr, include/hgx.h hgx_snapshot_*): write/read round trips
through libhgx.so, the header, the checksum, writer-side validation and the exporter's handle
table.  No GPU: the file entry points do no device work."""
import os
import struct

import numpy as np
import pytest

import kat_graphs as K


def _write(path, g, handles=None):
    from hypergraphdb_amd import write_snapshot
    write_snapshot(path, g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g.get("link_type"), handles)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_round_trip_random(tmp_path, seed):
    from hypergraphdb_amd import read_snapshot
    g = K.random_graph(np.random.default_rng(seed), 40 + 20 * seed, 30 + 10 * seed)
    p = str(tmp_path / "g.hgcsr")
    _write(p, g)
    f = read_snapshot(p)
    assert f["num_atoms"] == g["num_atoms"]
    for k in ("link_atom", "tgt_off", "tgt_idx", "link_type"):
        np.testing.assert_array_equal(f[k], g[k], err_msg=k)
    assert f["handles"] is None
    size = os.path.getsize(p)
    assert size % 64 == 0


def test_header_layout(tmp_path):
    """64-byte header: magic, version, flags, counts, handle width, checksum."""
    g = K.random_graph(np.random.default_rng(5), 20, 10)
    p = str(tmp_path / "g.hgcsr")
    _write(p, g)
    raw = open(p, "rb").read(64)
    magic, ver, flags, A, M, P, hb, _res, _ck = struct.unpack("<8sIIqqqIIQ", raw[:56])
    assert magic == b"HGXCSR1\0" and ver == 2 and flags == 1 and hb == 0
    assert (A, M, P) == (g["num_atoms"], len(g["link_atom"]), int(g["tgt_off"][-1]))
    # the link_atom section starts right after the header
    la = np.frombuffer(open(p, "rb").read()[64:64 + 4 * M], np.int32)
    np.testing.assert_array_equal(la, g["link_atom"])


def test_untyped_and_empty(tmp_path):
    from hypergraphdb_amd import read_snapshot, write_snapshot
    p = str(tmp_path / "e.hgcsr")
    write_snapshot(p, 5, np.zeros(0, np.int32), np.zeros(1, np.int64), np.zeros(0, np.int32))
    f = read_snapshot(p)
    assert f["num_atoms"] == 5 and len(f["link_atom"]) == 0 and f["tgt_off"].tolist() == [0]
    assert f["link_type"] is None
    g = K.random_graph(np.random.default_rng(9), 10, 6)
    write_snapshot(p, g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"])   # replaces the file
    f = read_snapshot(p)
    assert f["link_type"] is None
    np.testing.assert_array_equal(f["tgt_idx"], g["tgt_idx"])
    assert not os.path.exists(p + ".tmp")


def test_corruption_is_detected(tmp_path):
    from hypergraphdb_amd import HGXError, read_snapshot
    from hypergraphdb_amd import _lib
    g = K.random_graph(np.random.default_rng(3), 30, 20)
    p = str(tmp_path / "g.hgcsr")
    _write(p, g)
    data = bytearray(open(p, "rb").read())
    # one flipped bit in the target section
    bad = bytearray(data)
    bad[64 + 4 * len(g["link_atom"]) + 8 * (len(g["link_atom"]) + 1) + 3] ^= 0x10
    q = str(tmp_path / "bad.hgcsr")
    open(q, "wb").write(bytes(bad))
    with pytest.raises(HGXError, match="checksum") as e:
        read_snapshot(q)
    assert e.value.code == _lib.HGX_E_INVALID
    # a corrupted header count (num_atoms + 5: extra isolated atoms) in a file without a handle table
    # is caught by the checksum, which covers the header
    bad = bytearray(data)
    bad[16:24] = struct.pack("<q", g["num_atoms"] + 5)
    open(q, "wb").write(bytes(bad))
    with pytest.raises(HGXError, match="checksum"):
        read_snapshot(q)
    bad = bytearray(data)
    bad[44:48] = struct.pack("<I", 1)   # the reserved word
    open(q, "wb").write(bytes(bad))
    with pytest.raises(HGXError, match="checksum"):
        read_snapshot(q)
    # bad magic, wrong version, truncation, missing file
    bad = bytearray(data)
    bad[0:1] = b"X"
    open(q, "wb").write(bytes(bad))
    with pytest.raises(HGXError, match="magic"):
        read_snapshot(q)
    bad = bytearray(data)
    bad[8:12] = struct.pack("<I", 7)
    open(q, "wb").write(bytes(bad))
    with pytest.raises(HGXError, match="version") as e:
        read_snapshot(q)
    assert e.value.code == _lib.HGX_E_UNSUPPORTED
    open(q, "wb").write(bytes(data[: len(data) - 64]))
    with pytest.raises(HGXError, match="truncated"):
        read_snapshot(q)
    with pytest.raises(HGXError) as e:
        read_snapshot(str(tmp_path / "missing.hgcsr"))
    assert e.value.code == _lib.HGX_E_NOTFOUND


def test_writer_validates_rows(tmp_path):
    from hypergraphdb_amd import HGXError, write_snapshot
    p = str(tmp_path / "g.hgcsr")
    with pytest.raises(HGXError, match="ascending"):      # link rows out of rank order
        write_snapshot(p, 4, [2, 1], [0, 1, 2], [0, 0])
    with pytest.raises(HGXError, match="range"):          # target outside the rank space
        write_snapshot(p, 4, [1, 2], [0, 1, 2], [0, 9])
    with pytest.raises(HGXError, match="tgt_off"):
        write_snapshot(p, 4, [1, 2], [1, 1, 2], [0, 0])
    assert not os.path.exists(p)


def test_exporter_handle_table(tmp_path):
    """export_store ranks handles in byte order (UUID.java:364-376) and stores the rank-ordered
    handle bytes, so a reader maps ranks back to persistent handles."""
    from hypergraphdb_amd import export_store, read_snapshot
    from hypergraphdb_amd.snapshot import handle_bytes
    rng = np.random.default_rng(11)
    handles = [bytes(rng.integers(0, 256, 16, dtype=np.uint8)) for _ in range(12)]
    layouts = {handles[3]: (2, [handles[0], handles[1]]), handles[7]: (1, [handles[3], handles[5], handles[3]]),
               handles[9]: (0, [])}
    p = str(tmp_path / "x.hgcsr")
    ranks = export_store(p, handles, layouts)
    f = read_snapshot(p)
    assert f["handles"].shape == (12, 16)
    for h, r in ranks.items():
        assert bytes(f["handles"][r]) == handle_bytes(h)
    rows = sorted(layouts, key=lambda h: ranks[h])
    assert f["link_atom"].tolist() == [ranks[h] for h in rows]
    for r, h in enumerate(rows):
        t, tg = layouts[h]
        assert f["link_type"][r] == t
        assert f["tgt_idx"][f["tgt_off"][r]:f["tgt_off"][r + 1]].tolist() == [ranks[x] for x in tg]
    # int handles: 4-byte IntPersistentHandle form
    ints = [5, -3, 100, 7]
    ranks = export_store(p, ints, {100: (0, [5, -3]), 7: (1, [100])})
    f = read_snapshot(p)
    assert f["handles"].shape == (4, 4)
    assert [bytes(x) for x in f["handles"]] == [handle_bytes(h) for h in sorted(ints)]


def test_handle_table_must_be_uniform(tmp_path):
    from hypergraphdb_amd import write_snapshot
    with pytest.raises(ValueError):
        write_snapshot(str(tmp_path / "u.hgcsr"), 2, [], [0], [], None, [1, bytes(16)])
