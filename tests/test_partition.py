"""Host-side hash partition (hgx_shard_build, no device work): every part's tables against a
direct restatement of the partition rule, and the multi-process view over a gloo group."""
import os
import socket

import numpy as np
import pytest

import kat_graphs as K


def _shards(g, NP):
    from hypergraphdb_amd.partition import Shard
    return [Shard.build(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g.get("link_type"), NP, p)
            for p in range(NP)]


def _check_part(g, NP, p, d):
    A = g["num_atoms"]
    off, tg = np.asarray(g["tgt_off"]), np.asarray(g["tgt_idx"])
    lt = np.zeros(len(g["link_atom"]), np.int32) if g.get("link_type") is None else np.asarray(g["link_type"])
    local_rows = [r for r in range(len(g["link_atom"])) if any(int(t) % NP == p for t in tg[off[r]:off[r + 1]])]
    atoms = set()                                  # owned atoms without incidence get no local id
    for r in local_rows:
        atoms.update(int(t) for t in tg[off[r]:off[r + 1]])
    assert d["l2g"].tolist() == sorted(atoms)                  # local ids follow global order
    assert d["link_atom"].tolist() == [int(g["link_atom"][r]) for r in local_rows]
    assert d["link_type"].tolist() == [int(lt[r]) for r in local_rows]
    for i, r in enumerate(local_rows):                           # targets in local ids, layout order kept
        got = d["l2g"][d["tgt_idx"][d["tgt_off"][i]:d["tgt_off"][i + 1]]].tolist()
        assert got == tg[off[r]:off[r + 1]].tolist()
    gc = np.zeros(NP, np.int64)
    for a in atoms:
        if a % NP != p:
            gc[a % NP] += 1
    assert d["ghost_count"].tolist() == gc.tolist()


@pytest.mark.parametrize("NP", [1, 2, 3, 5, 8])
def test_shard_tables_random_graph(NP):
    rng = np.random.default_rng(100 + NP)
    g = K.random_graph(rng, 300, 500, max_arity=6, n_types=3)
    shards = _shards(g, NP)
    owned = []
    for p, s in enumerate(shards):
        d = s.export()
        _check_part(g, NP, p, d)
        owned.extend(int(a) for a in d["l2g"] if a % NP == p)
        assert s.n_owned == len(range(p, g["num_atoms"], NP))
    targets = sorted(set(np.asarray(g["tgt_idx"]).tolist()))
    assert sorted(owned) == targets                # every atom with incidence is owned exactly once
    # every link is held by each part owning one of its targets (replication <= arity)
    row_of = {int(a): r for r, a in enumerate(g["link_atom"])}
    held = np.zeros(len(g["link_atom"]), np.int64)
    for s in shards:
        for la in s.export()["link_atom"]:
            held[row_of[int(la)]] += 1
    off, tg = g["tgt_off"], np.asarray(g["tgt_idx"])
    for r in range(len(held)):
        assert held[r] == len({int(t) % NP for t in tg[off[r]:off[r + 1]]})
    for s in shards:
        s.close()


def test_shard_kat_graphs_and_power_law():
    from hypergraphdb_amd import synth
    for g in (K.queries_graph(), K.linkage_graph(), synth.hypergraph(2000, 6000, 2, 8, 2.1, 4, seed=5)):
        for NP in (2, 4):
            for p, s in enumerate(_shards(g, NP)):
                if g["num_atoms"] > 5000 and p > 0:
                    continue                                     # large graph: one part is enough here
                _check_part(g, NP, p, s.export())
                s.close()


def test_shard_errors():
    from hypergraphdb_amd import HGXError
    from hypergraphdb_amd.partition import Shard
    g = K.queries_graph()
    with pytest.raises(HGXError):
        Shard.build(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], None, 2, 2)
    bad = np.asarray(g["tgt_idx"]).copy()
    bad[0] = g["num_atoms"] + 5
    with pytest.raises(HGXError):
        Shard.build(g["num_atoms"], g["link_atom"], g["tgt_off"], bad, None, 2, 0)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    from hypergraphdb_amd import synth
    from hypergraphdb_amd.partition import Shard
    dist.init_process_group("gloo")
    g = synth.hypergraph(1500, 4000, 2, 6, 2.1, 2, seed=21)
    s = Shard.build(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"], world, rank)
    d = s.export()
    mine = {"owned": [int(a) for a in d["l2g"] if a % world == rank], "links": d["link_atom"].tolist(),
            "ghost_count": d["ghost_count"].tolist(), "l2g": d["l2g"].tolist()}
    views = [None] * world
    dist.all_gather_object(views, mine)
    if rank == 0:
        owned = sorted(a for v in views for a in v["owned"])
        ok = owned == sorted(set(g["tgt_idx"].tolist()))
        # rank p's ghosts owned by r == atoms of r that p must receive rows for
        for p in range(world):
            for r in range(world):
                n = sum(1 for a in views[p]["l2g"] if a % world == r and r != p)
                ok &= views[p]["ghost_count"][r] == n
        # a link is held by exactly the parts owning one of its targets
        off, tg = g["tgt_off"], g["tgt_idx"]
        for r in range(0, len(g["link_atom"]), 97):
            la = int(g["link_atom"][r])
            parts = {int(t) % world for t in tg[off[r]:off[r + 1]]}
            ok &= all((la in set(views[p]["links"])) == (p in parts) for p in range(world))
        q.put(bool(ok))
    dist.barrier()
    dist.destroy_process_group()


def test_partition_world2_gloo():
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    ok = q.get(timeout=240)
    for p in ps:
        p.join(timeout=60)
    assert ok
    assert all(p.exitcode == 0 for p in ps)
