"""Generates the committed golden fixtures of tests/golden/ (run in the build container only).

Every expected output comes from the pure-Python restatement oracle/pyref.py and is
cross-checked against the C restatement oracle/hgx_oracle.c before it is written; the script
refuses to write a fixture on any disagreement.  Inputs are the reference's own known-answer
test graphs (tests/kat_graphs.py), seeded random edge-case hypergraphs, and the config-1 graph of
SURVEY.md 8(d).  Usage:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]

import kat_graphs as K  # noqa: E402
import pyref  # noqa: E402
from oracle_ctypes import OracleGraph, algen  # noqa: E402


def pygraph(g):
    links = {}
    for r, la in enumerate(g["link_atom"].tolist()):
        links[la] = (int(g["link_type"][r]), g["tgt_idx"][g["tgt_off"][r]:g["tgt_off"][r + 1]].tolist())
    return pyref.Graph(list(range(g["num_atoms"])), links)


def ograph(g):
    return OracleGraph(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])


def py_bfs(pg, seed, maxd, mode, lt=None):
    P, S, R, RS = mode
    return pyref.bfs(pg, seed, maxd, link_type=lt, preceding=P, succeeding=S, reverse=R, source=RS)


def c_bfs(og, seed, maxd, mode, lt=-1):
    P, S, R, RS = mode
    l, a, d, _ = og.bfs(seed, -1 if maxd is None else maxd, algen(lt, P, S, R, RS))
    return list(zip(l.tolist(), a.tolist(), d.tolist()))


def agree_bfs(pg, og, seed, maxd, mode, lt):
    s1 = py_bfs(pg, seed, maxd, mode, None if lt < 0 else lt)
    s2 = c_bfs(og, seed, maxd, mode, lt)
    if s1 != s2:
        raise SystemExit(f"restatements disagree: seed {seed} maxd {maxd} mode {mode} lt {lt}")
    return s1


def graph_digest(g):
    import hashlib
    h = hashlib.sha256()
    for k in ("link_atom", "tgt_off", "tgt_idx"):
        h.update(np.ascontiguousarray(g[k]).tobytes())
    return h.hexdigest()


def pack_seq(seq):
    return np.array(seq, np.int32).reshape(-1, 3)


def main():
    out_json = {}
    # ---- KAT graphs ------------------------------------------------------------------
    for name, fn in [("linkage", K.linkage_graph), ("queries", K.queries_graph), ("pattern", K.pattern_graph),
                     ("compilation", K.compilation_graph)]:
        g = fn()
        pg, og = pygraph(g), ograph(g)
        entry = {k: (v.tolist() if isinstance(v, np.ndarray) else v) for k, v in g.items()}
        entry["bfs"] = {}
        for a in range(g["num_atoms"]):
            for mi, mode in enumerate(K.ALGEN_MODES):
                for maxd in (None, 1, 2):
                    seq = agree_bfs(pg, og, a, maxd, mode, -1)
                    entry["bfs"][f"{a}/{mi}/{maxd}"] = seq
        entry["incidence"] = {str(a): og.incidence(a).tolist() for a in range(g["num_atoms"])}
        for a in range(g["num_atoms"]):
            assert entry["incidence"][str(a)] == pg.inc[a]
        out_json[name] = entry
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(out_json, f, separators=(",", ":"))

    # ---- random edge-case graphs: BFS per mode + and-queries --------------------------
    rng = np.random.default_rng(20261015)
    arrays = {}
    for gi in range(12):
        g = K.random_graph(rng, int(rng.integers(5, 40)), int(rng.integers(3, 40)),
                           link_targets=bool(gi % 3), n_types=3)
        pg, og = pygraph(g), ograph(g)
        for k in ("link_atom", "tgt_off", "tgt_idx", "link_type"):
            arrays[f"g{gi}_{k}"] = g[k]
        arrays[f"g{gi}_A"] = np.array([g["num_atoms"]], np.int64)
        seqs, keys = [], []
        for s in range(min(g["num_atoms"], 8)):
            seed = int(rng.integers(0, g["num_atoms"]))
            mi = int(rng.integers(0, len(K.ALGEN_MODES)))
            lt = int(rng.integers(-1, 3))
            maxd = [None, 1, 2, 3][int(rng.integers(0, 4))]
            seq = agree_bfs(pg, og, seed, maxd, K.ALGEN_MODES[mi], lt)
            keys.append([seed, mi, lt, -1 if maxd is None else maxd, len(seq)])
            seqs += seq
        arrays[f"g{gi}_bfs_keys"] = np.array(keys, np.int32)
        arrays[f"g{gi}_bfs_seq"] = pack_seq(seqs)
        # and-queries
        qkeys, qres = [], []
        for _ in range(12):
            t = int(rng.integers(-1, 3))
            inc = [int(x) for x in rng.integers(0, g["num_atoms"], int(rng.integers(0, 3)))]
            m = int(rng.integers(-1, 4))
            pat = None if m < 0 else [int(x) if rng.random() < 0.7 else -1 for x in rng.integers(0, g["num_atoms"], m)]
            r_py = pyref.and_query(pg, None if t < 0 else t, inc, pat)
            r_c = og.and_query(t, inc, pat)
            r_set = og.and_query(t, inc, pat, zigzag=False)
            if r_py is None:
                assert r_c is None and r_set is None
                continue
            if not (list(r_py) == r_c.tolist() == r_set.tolist()):
                raise SystemExit(f"and-query restatements disagree on g{gi}: {t} {inc} {pat}")
            qkeys.append([t, len(inc), -1 if pat is None else len(pat), len(r_py)] + inc + (pat or []))
            qres += list(r_py)
        arrays[f"g{gi}_q_keys"] = np.array(json.dumps(qkeys))
        arrays[f"g{gi}_q_res"] = np.array(qres, np.int32)
    np.savez_compressed(os.path.join(HERE, "random_small.npz"), **arrays)

    # ---- config 1: per-seed per-depth sets ------------------------------
    from hypergraphdb_amd import synth
    g = synth.config1()
    pg, og = pygraph(g), ograph(g)
    lv_off, lv_ids = [0], []
    for s in g["seeds"].tolist():
        seq = agree_bfs(pg, og, s, 3, K.ALGEN_MODES[0], -1)
        levels = pyref.per_depth_sets(seq, s, 4)
        for lv in levels:
            lv_ids += lv
            lv_off.append(len(lv_ids))
    # the graph itself is regenerated by hypergraphdb_amd.synth.config1() in the tests and pinned
    # here by its SHA-256 (keeps the fixture small)
    np.savez_compressed(os.path.join(HERE, "config1.npz"), num_atoms=np.array([g["num_atoms"]]),
                        graph_sha256=np.array(graph_digest(g)), seeds=g["seeds"],
                        level_off=np.array(lv_off, np.int64), level_ids=np.array(lv_ids, np.int32))
    print("fixtures written:", sorted(os.listdir(HERE)))


if __name__ == "__main__":
    main()
