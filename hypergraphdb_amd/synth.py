"""Synthetic inputs of SURVEY.md section 8(d) (configs 1-5), built by the native generators in
csrc/hgx_gen.c.  Atom ids follow IntHandleFactory add order: nodes 0..N-1, then links."""
from __future__ import annotations

import numpy as np

from ._lib import gen_lib, ptr


def hypergraph(n_nodes, n_links, arity_lo, arity_hi, gamma=0.0, n_types=1, seed=1):
    """Returns dict(num_atoms, link_atom, tgt_off, tgt_idx, link_type)."""
    G = gen_lib()
    off = np.zeros(n_links + 1, np.int64)
    P = G.hgx_gen_hypergraph_offsets(n_links, arity_lo, arity_hi, seed, ptr(off))
    tgt = np.empty(max(P, 1), np.int32)
    lt = np.zeros(max(n_links, 1), np.int32)
    rc = G.hgx_gen_hypergraph_fill(n_nodes, n_links, arity_lo, arity_hi, float(gamma), n_types, seed, ptr(off),
                                   ptr(tgt), ptr(lt))
    if rc != 0:
        raise RuntimeError("generator failed")
    return dict(num_atoms=n_nodes + n_links, n_nodes=n_nodes,
                link_atom=np.arange(n_nodes, n_nodes + n_links, dtype=np.int32),
                tgt_off=off, tgt_idx=tgt[:P], link_type=lt[:n_links])


def permutation_prefix(n, k, seed):
    out = np.empty(k, np.int32)
    gen_lib().hgx_gen_permutation_prefix(n, k, seed, ptr(out))
    return out


def sources(g, k, seed):
    out = np.empty(k, np.int32)
    rc = gen_lib().hgx_gen_sources(g["n_nodes"], len(g["tgt_idx"]), ptr(g["tgt_idx"]), k, seed, ptr(out))
    if rc != 0:
        raise RuntimeError("not enough nodes with deg >= 1")
    return out


def config1(scale=1.0):
    """100K nodes + 100K links, arity U{2,3,4}, uniform distinct targets, seed 1; 64 sources =
    first 64 of a seed-2 permutation of node ids; depth 3."""
    n = max(int(100_000 * scale), 16)
    g = hypergraph(n, n, 2, 4, 0.0, 1, seed=1)
    g["seeds"] = permutation_prefix(n, min(64, n), 2)
    g["depth"] = 3
    return g


def config2(scale=1.0, n_sources=1024):
    """10M nodes, 40M links, arity U{2..8}, Chung-Lu gamma 2.1, seed 42; 1024 sources over nodes
    with deg >= 1 (seed 7); depth 4."""
    n, m = max(int(10_000_000 * scale), 64), max(int(40_000_000 * scale), 64)
    g = hypergraph(n, m, 2, 8, 2.1, 1, seed=42)
    g["seeds"] = sources(g, n_sources, 7)
    g["depth"] = 4
    return g


def config3(scale=1.0, n_queries=10_000):
    """50M links over 10M nodes, arity U{3..6}, 64 link types (seed 43), Chung-Lu gamma 2.1;
    queries hg.and(hg.type(T), hg.incident(a), hg.orderedLink(x, ANY, y)) (seed 44, 10% negatives)."""
    n, m = max(int(10_000_000 * scale), 64), max(int(50_000_000 * scale), 64)
    g = hypergraph(n, m, 3, 6, 2.1, 64, seed=43)
    q = {k: np.empty(n_queries, np.int32) for k in ("type", "a", "x", "y", "row")}
    gen_lib().hgx_gen_queries(n, m, ptr(g["tgt_off"]), ptr(g["tgt_idx"]), ptr(g["link_type"]), n_queries, 0.10, 44,
                              ptr(q["type"]), ptr(q["a"]), ptr(q["x"]), ptr(q["y"]), ptr(q["row"]))
    g["queries"] = q
    return g


def config4(scale=1.0, n_sources=1024):
    """100M nodes, 200M links, arity U{2..8} (P ~ 1.0B incidences), Chung-Lu gamma 2.1, seed 45;
    1024 sources over nodes with deg >= 1 (seed 7); depth 4.  Hash-partitioned over the GPUs."""
    n, m = max(int(100_000_000 * scale), 64), max(int(200_000_000 * scale), 64)
    g = hypergraph(n, m, 2, 8, 2.1, 1, seed=45)
    g["seeds"] = sources(g, n_sources, 7)
    g["depth"] = 4
    return g


def config5(scale=1.0, n_sources=1024, subsumes_type=1, noise_type=2):
    """5M classes; class i > 0 gets 1-3 HGSubsumes(parent, i) links with preferential parents
    (seed 46) + 5M noise arity-2 links of another type; 1024 sources uniform over classes."""
    C_ = max(int(5_000_000 * scale), 16)
    noise = max(int(5_000_000 * scale), 1)
    G = gen_lib()
    M = G.hgx_gen_ontology(C_, noise, 46, subsumes_type, noise_type, None, None)
    tgt = np.empty(2 * M, np.int32)
    lt = np.empty(M, np.int32)
    G.hgx_gen_ontology(C_, noise, 46, subsumes_type, noise_type, ptr(tgt), ptr(lt))
    g = dict(num_atoms=C_ + M, n_nodes=C_, link_atom=np.arange(C_, C_ + M, dtype=np.int32),
             tgt_off=np.arange(0, 2 * M + 1, 2, dtype=np.int64), tgt_idx=tgt, link_type=lt)
    g["seeds"] = permutation_prefix(C_, min(n_sources, C_), 47)
    g["subsumes_type"] = subsumes_type
    return g
