"""Host-side vertex-cut partition (hgx_partition_plan / hgx_shard_build, no device work): the
placement (deterministic, pin-balanced, fewer remote holders than a random placement), every part's
tables against a direct restatement of the partition rule, the exchange tables (owner and holder
local ids) and the multi-process view over a gloo group (every rank computes the same plan)."""
import os
import socket

import numpy as np
import pytest

import kat_graphs as K


def _plan(g, NP):
    from hypergraphdb_amd.partition import partition_plan
    return partition_plan(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g.get("link_type"), NP)


def _shards(g, NP, plan=None):
    from hypergraphdb_amd.partition import Shard
    plan = _plan(g, NP) if plan is None else plan
    return plan, [Shard.build(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g.get("link_type"), NP, p,
                              plan) for p in range(NP)]


def _holders(g, plan, NP):
    off, tg = np.asarray(g["tgt_off"]), np.asarray(g["tgt_idx"])
    hold = [set() for _ in range(g["num_atoms"])]
    for r in range(len(g["link_atom"])):
        for t in tg[off[r]:off[r + 1]]:
            hold[int(t)].add(int(plan[r]))
    return hold


def _check(g, NP, plan, shards):
    off, tg = np.asarray(g["tgt_off"]), np.asarray(g["tgt_idx"])
    lt = np.zeros(len(g["link_atom"]), np.int32) if g.get("link_type") is None else np.asarray(g["link_type"])
    hold = _holders(g, plan, NP)
    ds = [s.export() for s in shards]
    xs = [s.exchange_tables() for s in shards]
    owner = {}
    for p, (s, d, x) in enumerate(zip(shards, ds, xs)):
        rows = [r for r in range(len(g["link_atom"])) if plan[r] == p]
        assert d["link_atom"].tolist() == [int(g["link_atom"][r]) for r in rows]
        assert d["link_type"].tolist() == [int(lt[r]) for r in rows]
        atoms = sorted({int(t) for r in rows for t in tg[off[r]:off[r + 1]]})
        assert d["l2g"].tolist() == atoms                          # local ids follow global order
        for i, r in enumerate(rows):                               # targets in local ids, layout order kept
            assert d["l2g"][d["tgt_idx"][d["tgt_off"][i]:d["tgt_off"][i + 1]]].tolist() == tg[off[r]:off[r + 1]].tolist()
        n_owned = 0
        for i, v in enumerate(d["l2g"].tolist()):
            assert p in hold[v]
            if x["xo_part"][i] < 0:                                 # owned here
                n_owned += 1
                assert v not in owner
                owner[v] = p
                others = sorted(hold[v] - {p})
                b, e = x["bc_off"][i], x["bc_off"][i + 1]
                assert x["bc_part"][b:e].tolist() == others
                for q, lid in zip(x["bc_part"][b:e], x["bc_lid"][b:e]):
                    assert ds[q]["l2g"][lid] == v                   # the holder's local id of v
            else:
                o, lid = int(x["xo_part"][i]), int(x["xo_lid"][i])
                assert o != p and o in hold[v] and ds[o]["l2g"][lid] == v
                assert x["bc_off"][i + 1] == x["bc_off"][i]
        assert s.n_owned == n_owned
    present = sorted(v for v in range(g["num_atoms"]) if hold[v])
    assert sorted(owner) == present                                # every present atom owned exactly once
    for p in range(NP):                                            # reduce records p -> q == broadcast q -> p
        for q in range(NP):
            assert ds[p]["ghost_count"][q] == xs[q]["bc_count"][p]


@pytest.mark.parametrize("NP", [1, 2, 3, 5, 8])
def test_vertex_cut_tables_random_graph(NP):
    rng = np.random.default_rng(100 + NP)
    g = K.random_graph(rng, 300, 500, max_arity=6, n_types=3)
    plan, shards = _shards(g, NP)
    assert plan.min() >= 0 and plan.max() < NP
    _check(g, NP, plan, shards)
    for s in shards:
        s.close()


def test_plan_deterministic_balanced_and_better_than_random():
    from hypergraphdb_amd import synth
    g = synth.hypergraph(20000, 60000, 2, 8, 2.1, 1, seed=5)
    NP = 8
    p1, p2 = _plan(g, NP), _plan(g, NP)
    assert np.array_equal(p1, p2)
    ar = np.diff(g["tgt_off"])
    load = np.bincount(p1, weights=ar, minlength=NP)
    assert load.max() <= 1.02 * ar.sum() / NP + 64 + ar.max()     # the pin-balance cap
    # remote holders (holders beyond the owner) per present atom: greedy vs random placement
    def remote(plan):
        off, tg = g["tgt_off"], g["tgt_idx"]
        part_of_pin = np.repeat(plan, ar)
        pairs = np.unique(tg.astype(np.int64) * NP + part_of_pin)
        present = len(np.unique(tg))
        return (len(pairs) - present) / present
    rnd = np.random.default_rng(1).integers(0, NP, len(p1)).astype(np.int32)
    assert remote(p1) < 0.75 * remote(rnd), (remote(p1), remote(rnd))


def test_vertex_cut_kat_graphs_and_power_law():
    from hypergraphdb_amd import synth
    for g in (K.queries_graph(), K.linkage_graph(), synth.hypergraph(2000, 6000, 2, 8, 2.1, 4, seed=5)):
        for NP in (2, 4):
            plan, shards = _shards(g, NP)
            _check(g, NP, plan, shards)
            for s in shards:
                s.close()


def test_shard_errors():
    from hypergraphdb_amd import HGXError
    from hypergraphdb_amd.partition import Shard, partition_plan
    g = K.queries_graph()
    plan = _plan(g, 2)
    with pytest.raises(HGXError):
        Shard.build(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], None, 2, 2, plan)
    with pytest.raises(HGXError, match="placement"):
        Shard.build(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], None, 2, 0, plan + 5)
    bad = np.asarray(g["tgt_idx"]).copy()
    bad[0] = g["num_atoms"] + 5
    with pytest.raises(HGXError):
        Shard.build(g["num_atoms"], g["link_atom"], g["tgt_off"], bad, None, 2, 0, plan)
    with pytest.raises(HGXError):
        partition_plan(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], None, 65)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    from hypergraphdb_amd import synth
    from hypergraphdb_amd.partition import Shard, partition_plan
    dist.init_process_group("gloo")
    g = synth.hypergraph(1500, 4000, 2, 6, 2.1, 2, seed=21)
    plan = partition_plan(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"], world)
    s = Shard.build(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"], world, rank, plan)
    d, x = s.export(), s.exchange_tables()
    mine = {"plan": plan.tolist(), "l2g": d["l2g"].tolist(), "links": d["link_atom"].tolist(),
            "owned": [int(v) for i, v in enumerate(d["l2g"]) if x["xo_part"][i] < 0],
            "ghost_count": d["ghost_count"].tolist(), "bc_count": x["bc_count"].tolist()}
    views = [None] * world
    dist.all_gather_object(views, mine)
    if rank == 0:
        ok = all(v["plan"] == views[0]["plan"] for v in views)     # every rank computed the same plan
        owned = sorted(a for v in views for a in v["owned"])
        ok &= owned == sorted(set(g["tgt_idx"].tolist()))
        ok &= sorted(a for v in views for a in v["links"]) == g["link_atom"].tolist()   # each link once
        for p in range(world):
            for r in range(world):
                ok &= views[p]["ghost_count"][r] == views[r]["bc_count"][p]
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
