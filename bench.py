#!/usr/bin/env python3
"""Benchmark: hyperedge TEPS of batched multi-source BFS (+ pattern-match queries/sec).

Workload (BASELINE.json configs[1]): config 2 -- 10M nodes, 40M links, arity
U{2..8}, Chung-Lu gamma 2.1, 1024-source BFS to depth 4 on one MI355X.  A step = one
hgx_bfs_batch over the 1024 sources with the CSR resident in HBM (all per-depth visited sets
materialised on the device).  Secondary: config 3, one step = one hgx_pattern_batch of 10,000
hg.and(hg.type(T), hg.incident(a), hg.orderedLink(x, ANY, y)) queries over 50M typed links.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): the sources
are independent units; every rank holds a replica of the snapshot and runs its own 1024-source
batch (weak scaling, no data-path collective).  torch.distributed is used only for the barrier
and the max-over-ranks of the elapsed time.

The CPU baseline is the C restatement of the reference path (oracle/, test infrastructure) timed
on the host cores on a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def log(msg):
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def pmc_traffic(kernel, workload):
    """HBM bytes per launch from a committed rocprofv3 PMC summary (profiles/pmc_<workload>.json,
    written by tools/pmc_summary.py with the gfx950 FETCH_SIZE correction), or None."""
    p = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    if not os.path.exists(p):
        return None
    try:
        d = json.load(open(p))
        return d.get("kernels", {}).get(kernel, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


def roofline(stats_list, workload):
    """Dominant kernel of the BFS step: achieved = algorithmic bytes / device time (HIP events)."""
    from hypergraphdb_amd._lib import KERNELS
    tot = {k: {"ms": 0.0, "bytes": 0.0, "launches": 0} for k in KERNELS}
    for st in stats_list:
        for k, v in st["kernels"].items():
            tot[k]["ms"] += v["ms"]
            tot[k]["bytes"] += v["bytes"]
            tot[k]["launches"] += v["launches"]
    dom = max(tot, key=lambda k: tot[k]["ms"])
    t = tot[dom]
    achieved = t["bytes"] / (t["ms"] / 1e3) / 1e9 if t["ms"] > 0 else 0.0
    traffic = pmc_traffic(dom, workload)
    return {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "bytes_per_launch": t["bytes"] / max(t["launches"], 1),
            "avg_launch_ms": t["ms"] / max(t["launches"], 1), "launches": t["launches"]}, tot


def cpu_bfs_baseline(g, seeds, depth, budget_s):
    """C restatement (oracle/) of HGBreadthFirstTraversal + DefaultALGenerator, OpenMP over seeds."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle_ctypes import OracleGraph
    threads = int(os.environ.get("HGX_CPU_THREADS", min(16, os.cpu_count() or 1)))
    t0 = time.time()
    orc = OracleGraph(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    log(f"cpu baseline: host snapshot built in {time.time() - t0:.1f}s; {threads} threads")
    # one traversal per thread, each stopped after budget_s (a bounded sample of the same workload:
    # the rate is the reference path's edge rate over the first budget_s of every traversal)
    batch = np.asarray(seeds[:threads], np.int32)
    tm = {}
    _, tr = orc.bfs_many(batch, depth, depth + 1, nthreads=threads, time_budget_s=budget_s, timing=tm)
    elapsed = tm["elapsed_s"]
    trav = int(tr.sum())
    del orc
    return {"value": trav / elapsed, "unit": "TEPS", "cores": threads, "kind": "port",
            "sample": f"{len(batch)} of the {len(seeds)} config-2 sources, depth {depth}, one traversal per thread "
                      f"(C restatement of HGBreadthFirstTraversal/DefaultALGenerator), each stopped after "
                      f"{budget_s:.0f}s; {trav:.3e} hyperedges in {elapsed:.1f}s",
            "seconds": round(elapsed, 2)}


def cpu_query_baseline(g, qs, budget_s):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle_ctypes import OracleGraph
    threads = int(os.environ.get("HGX_CPU_THREADS", min(16, os.cpu_count() or 1)))
    orc = OracleGraph(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    n_done, elapsed, i, step = 0, 0.0, 0, max(threads * 8, 64)
    while elapsed < budget_s and i < len(qs["type"]):
        sl = slice(i, i + step)
        t = qs["type"][sl]
        n = len(t)
        inc_off = np.arange(n + 1, dtype=np.int64)
        pat_off = np.arange(0, 3 * n + 1, 3, dtype=np.int64)
        pat = np.stack([qs["x"][sl], np.full(n, -1, np.int32), qs["y"][sl]], 1).reshape(-1)
        t1 = time.time()
        orc.and_query_many(t, inc_off, qs["a"][sl], pat_off, pat, np.ones(n, np.int32), nthreads=threads)
        elapsed += time.time() - t1
        n_done += n
        i += step
    del orc
    return {"value": n_done / elapsed, "unit": "queries/s", "cores": threads, "kind": "port",
            "sample": f"{n_done} of the {len(qs['type'])} config-3 queries (C restatement of AndToQuery + "
                      f"ZigZagIntersectionResult + OrderedLinkCondition), {elapsed:.1f}s",
            "seconds": round(elapsed, 2)}


def _kernel_roof(stats_list):
    tot = {}
    for st in stats_list:
        for k, v in st["kernels"].items():
            t = tot.setdefault(k, {"ms": 0.0, "bytes": 0.0, "launches": 0})
            t["ms"] += v["ms"]
            t["bytes"] += v["bytes"]
            t["launches"] += v["launches"]
    dom = max(tot, key=lambda k: tot[k]["ms"])
    t = tot[dom]
    ach = t["bytes"] / (t["ms"] / 1e3) / 1e9 if t["ms"] > 0 else 0.0
    return {"bound": "hbm", "kernel": dom, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "avg_launch_ms": round(t["ms"] / max(t["launches"], 1), 4)}


def run_config4(args, ctx, barrier_sync, result):
    """Config 4 (1B incidences) in its two multi-GPU forms:
      replicated  -- every GPU holds the whole snapshot (compacted one-part shard, ~16 GB of CSR)
                     and runs its own 1024-source batch (weak scaling: throughput of the batch
                     workload, no data-path collective);
      partitioned -- the snapshot is hash-partitioned over the N GPUs (owner = atom % N) and the
                     same 1024 sources run together, one RCCL all-to-all of ghost rows per level
                     (strong scaling; the path for graphs beyond one GPU's 288 GB).
    Fills result[...] in place so a watchdog can still report what finished."""
    from hypergraphdb_amd import dist as hdist
    from hypergraphdb_amd import synth
    from hypergraphdb_amd.partition import RcclComm, Shard, ShardSnapshot, pbfs_batch, pbfs_batch_group
    rank, world, local = ctx.rank, ctx.world, ctx.device
    t0 = time.time()
    g = synth.config4(scale=args.c4_scale, n_sources=args.sources)
    log(f"rank {rank}: config4 generated in {time.time() - t0:.1f}s: A={g['num_atoms']} P={len(g['tgt_idx'])}")
    wl = (f"config4: 100M nodes / 200M links (1.0B incidences), Chung-Lu gamma 2.1, {args.sources}-source BFS "
          f"depth {args.depth}" if args.c4_scale == 1.0 else f"config4 at scale {args.c4_scale}")

    def timed(run, n_steps):
        barrier_sync()
        t1 = time.perf_counter()
        st = []
        for _ in range(n_steps):
            r = run()
            st.append(r.stats(accounting=False))
            r.close()
        barrier_sync()
        return ctx.max(time.perf_counter() - t1), st

    # replicated snapshot, one 1024-source batch per GPU
    t0 = time.time()
    sh = Shard.build(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"], 1, 0)
    snap = ShardSnapshot(sh, local)
    log(f"rank {rank}: config4 replica (one part, {sh.n_local} atoms with incidence) on device in "
        f"{time.time() - t0:.1f}s")
    sh.close()
    snap.set_timing(True)
    mine = hdist.rank_sources(g, args.sources, rank)
    for _ in range(max(args.warmup, 1)):
        r = pbfs_batch_group([snap], mine, args.depth)
        acct = r.parts[0].stats(accounting=True)
        r.close()
    dt, st = timed(lambda: pbfs_batch_group([snap], mine, args.depth).parts[0], args.steps)
    edges = ctx.sum(acct["traversed_edges"] * args.steps)
    result["replicated"] = {
        "metric": "hyperedge TEPS", "value": edges / dt, "unit": "TEPS", "scaling": "weak",
        "ms_per_step": round(dt / args.steps * 1e3, 3), "workload": wl, "n_gpus": world,
        "parallelism": f"snapshot replicated on {world} GPU(s), {args.sources} sources per GPU",
        "traversed_edges_per_step": edges / args.steps, "roofline": _kernel_roof(st)}
    log(f"rank {rank}: config4 replicated {edges / dt:.3e} TEPS, {dt / args.steps * 1e3:.1f} ms/step")
    snap.close()
    del snap
    if world == 1:
        result["partitioned"] = dict(result["replicated"], scaling="strong",
                                     parallelism="one part: the hash partition degenerates to the replica")
        return
    # hash partition over the ranks, RCCL all-to-all per level, the same 1024 sources everywhere
    seeds = g["seeds"]
    t0 = time.time()
    sh = Shard.build(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"], world, rank)
    info = {"local_atoms": sh.n_local, "local_links": sh.n_links, "local_pins": sh.n_pins}
    snap = ShardSnapshot(sh, local)
    sh.close()
    del g
    snap.set_timing(True)
    comm = RcclComm.create(world, rank, local, broadcast=ctx.broadcast_bytes)
    log(f"rank {rank}: config4 part {rank}/{world} on device + RCCL comm in {time.time() - t0:.1f}s {info}")
    for _ in range(max(args.warmup, 1)):
        r = pbfs_batch(snap, comm, seeds, args.depth)
        acct = r.stats(accounting=True)
        r.close()
    dt, st = timed(lambda: pbfs_batch(snap, comm, seeds, args.depth), args.steps)
    edges = ctx.sum(acct["traversed_edges"] * args.steps)
    xbytes = ctx.sum(sum(s["bytes_exchanged"] for s in st)) / args.steps
    xms = ctx.max(sum(s["ms_exchange"] for s in st) / args.steps)
    result["partitioned"] = {
        "metric": "hyperedge TEPS", "value": edges / dt, "unit": "TEPS", "scaling": "strong",
        "ms_per_step": round(dt / args.steps * 1e3, 3), "workload": wl, "n_gpus": world,
        "parallelism": f"hash partition over {world} GPUs (owner = atom % {world}), RCCL all-to-all per level",
        "exchange_bytes_per_step": xbytes, "exchange_ms_per_step": round(xms, 3),
        "rank0_part": info, "roofline": _kernel_roof(st)}
    log(f"rank {rank}: config4 partitioned {edges / dt:.3e} TEPS, {dt / args.steps * 1e3:.1f} ms/step, "
        f"exchange {xbytes / 1e9:.2f} GB/step")
    comm.close()
    snap.close()


def run_config5(args, ctx, barrier_sync):
    """Config 5: hg.subsumed(G) / hg.subsumes(S) closures (unbounded BFS over HGSubsumes links only,
    C/query/cond2qry/ToQueryMap.java:282-370) for 1024 classes of a 5M-class ontology, both
    directions in one step.  Weak scaling: every GPU runs its own 1024 classes."""
    import hypergraphdb_amd as H
    from hypergraphdb_amd import AtomTypeCondition, DefaultALGenerator, synth
    rank, world = ctx.rank, ctx.world
    t0 = time.time()
    g = synth.config5(scale=args.c5_scale, n_sources=args.sources)
    if rank > 0:
        g["seeds"] = synth.permutation_prefix(g["n_nodes"], args.sources, 47 + 1000 * rank)
    snap = H.HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"],
                                device=ctx.device)
    snap.set_timing(True)
    T = g["subsumes_type"]
    gens = [DefaultALGenerator(snap, AtomTypeCondition(T), None, False, True, rev) for rev in (False, True)]
    log(f"rank {rank}: config5 ({g['n_nodes']} classes, {len(g['link_atom'])} links) ready in {time.time() - t0:.1f}s")
    trav, closure = 0.0, 0
    for _ in range(max(args.warmup, 1)):
        for gen in gens:
            r = H.bfs_batch(snap, g["seeds"], None, gen)
            st = r.stats(accounting=True)
            trav += st["traversed_edges"]
            closure += int(r.counts()[:, 1:].sum())
            r.close()
    trav /= max(args.warmup, 1)
    closure //= max(args.warmup, 1)
    barrier_sync()
    t1 = time.perf_counter()
    sts = []
    for _ in range(args.steps):
        for gen in gens:
            r = H.bfs_batch(snap, g["seeds"], None, gen)
            sts.append(r.stats(accounting=False))
            r.close()
    barrier_sync()
    dt = ctx.max(time.perf_counter() - t1)
    edges = ctx.sum(trav * args.steps)
    out = {"metric": "hyperedge TEPS (subsumption closures)", "value": edges / dt, "unit": "TEPS",
           "closures_per_s": ctx.sum(2 * len(g["seeds"]) * args.steps) / dt, "scaling": "weak",
           "ms_per_step": round(dt / args.steps * 1e3, 3), "levels": max(s["n_levels_expanded"] for s in sts),
           "closure_atoms_per_step": closure,
           "workload": (f"config5: {g['n_nodes']} classes, HGSubsumes DAG + noise links, {len(g['seeds'])} classes x "
                        "{subsumed, subsumes}, unbounded depth"),
           "roofline": _kernel_roof(sts)}
    log(f"rank {rank}: config5 {out['value']:.3e} TEPS, {out['closures_per_s']:.1f} closures/s, "
        f"{out['ms_per_step']} ms/step, {out['levels']} levels")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        from oracle_ctypes import OracleGraph, algen
        threads = int(os.environ.get("HGX_CPU_THREADS", min(16, os.cpu_count() or 1)))
        orc = OracleGraph(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
        tm, n, tr, el = {}, 0, 0, 0.0
        for rev in (False, True):
            batch = g["seeds"]   # every closure of the step (bounded by the time budget)
            _, t_ = orc.bfs_many(batch, -1, 4096, algen(T, False, True, rev, False), nthreads=threads,
                                 time_budget_s=args.cpu_budget / 2, timing=tm)
            tr += int(t_.sum())
            el += tm["elapsed_s"]
            n += len(batch)
        out["cpu_baseline"] = {"value": tr / el, "unit": "TEPS", "cores": threads, "kind": "port",
                               "sample": f"{n} closures (C restatement of the subsumption BFS), {el:.1f}s",
                               "seconds": round(el, 2)}
        del orc
    snap.close()
    return out


_JSON_FD = None


def claim_stdout():
    """Native libraries write to fd 1 (gloo's peer-connection notes, RCCL's version banner): route
    fd 1 to stderr for the whole run and keep the original stdout for the one JSON line."""
    global _JSON_FD
    sys.stdout.flush()
    _JSON_FD = os.dup(1)
    os.dup2(2, 1)


def emit(line):
    data = (json.dumps(line) + "\n").encode()
    if _JSON_FD is None:
        sys.stdout.write(data.decode())
        sys.stdout.flush()
        return
    sys.stdout.flush()
    while data:
        data = data[os.write(_JSON_FD, data):]


def main():
    claim_stdout()
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--scale", type=float, default=1.0, help="fraction of the config-2/3 sizes (1.0 = full)")
    ap.add_argument("--sources", type=int, default=1024)
    ap.add_argument("--depth", type=int, default=4)
    ap.add_argument("--no-queries", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=15.0, help="seconds of CPU-baseline work per metric")
    ap.add_argument("--no-config4", action="store_true", help="skip the config-4 (1B incidences) legs")
    ap.add_argument("--no-config5", action="store_true", help="skip the config-5 subsumption leg")
    ap.add_argument("--c5-scale", type=float, default=1.0, help="fraction of the config-5 size")
    ap.add_argument("--c4-scale", type=float, default=1.0, help="fraction of the config-4 size")
    ap.add_argument("--c4-timeout", type=float, default=420.0,
                    help="seconds after which the config-4 legs are abandoned (the line is still printed)")
    args = ap.parse_args()

    from hypergraphdb_amd import dist as hdist
    from hypergraphdb_amd._lib import device_synchronize

    # one process per GPU; only the barrier and scalar max/sum cross processes (gloo, CPU)
    ctx = hdist.init_from_env("gloo")
    rank, world, local = ctx.rank, ctx.world, ctx.device

    def barrier_sync():
        ctx.barrier()
        device_synchronize(local)   # hipDeviceSynchronize (the torch.cuda.synchronize equivalent)

    max_over_ranks, sum_over_ranks = ctx.max, ctx.sum

    import hypergraphdb_amd as H
    from hypergraphdb_amd import synth

    # ---------------- config 2: batched BFS ----------------
    t0 = time.time()
    g = synth.config2(scale=args.scale, n_sources=args.sources)
    g["seeds"] = hdist.rank_sources(g, args.sources, rank)   # weak scaling: every rank its own sources
    log(f"rank {rank}: config2 generated in {time.time() - t0:.1f}s: A={g['num_atoms']} M={len(g['link_atom'])} "
        f"P={len(g['tgt_idx'])}")
    t0 = time.time()
    snap = H.HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"],
                                device=local)
    log(f"rank {rank}: snapshot on device {local} in {time.time() - t0:.1f}s (I={snap.num_incidences})")
    snap.set_timing(True)
    acct = None
    for w in range(args.warmup):
        res = H.bfs_batch(snap, g["seeds"], args.depth)
        if acct is None:
            acct = res.stats(accounting=True)     # TEPS numerator / |U_d| (deterministic per batch)
            log(f"rank {rank}: levels |U_d|={acct['union_frontier']} traversed={acct['traversed_edges']:.3e}")
        res.close()
        log(f"rank {rank}: warmup {w} done")
    if acct is None:
        res = H.bfs_batch(snap, g["seeds"], args.depth)
        acct = res.stats(accounting=True)
        res.close()
    stats = []
    barrier_sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = H.bfs_batch(snap, g["seeds"], args.depth)
        stats.append(res.stats(accounting=False))
        res.close()
    barrier_sync()
    dt = max_over_ranks(time.perf_counter() - t0)
    edges_total = sum_over_ranks(acct["traversed_edges"] * args.steps)
    teps = edges_total / dt
    roof, per_kernel = roofline(stats, "config2")
    ms_dev = sum(s["ms_total"] for s in stats) / len(stats)
    log(f"rank {rank}: {args.steps} steps in {dt:.3f}s -> {teps:.3e} TEPS; device ms/step {ms_dev:.2f}; "
        f"dominant {roof['kernel']} {roof['achieved']} GB/s")
    snap.close()
    del snap

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_bfs_baseline(g, g["seeds"], args.depth, args.cpu_budget)
        log(f"cpu baseline {cpu['value']:.3e} TEPS on {cpu['cores']} threads")
    del g

    # ---------------- config 3: pattern queries ----------------
    pattern = None
    if not args.no_queries:
        t0 = time.time()
        g3 = synth.config3(scale=args.scale, n_queries=10_000)
        Q = g3["queries"]
        log(f"rank {rank}: config3 generated in {time.time() - t0:.1f}s")
        snap3 = H.HyperGraphSnapshot(g3["num_atoms"], g3["link_atom"], g3["tgt_off"], g3["tgt_idx"],
                                     g3["link_type"], device=local)
        snap3.set_timing(True)
        from hypergraphdb_amd.query import pattern_batch_arrays
        nq = len(Q["type"])
        # hg.and(hg.type(T), hg.incident(a), hg.orderedLink(x, hg.anyHandle(), y)) as one packed batch
        packed = (Q["type"], np.arange(nq + 1, dtype=np.int64), Q["a"], np.ones(nq, np.int32),
                  np.arange(0, 3 * nq + 1, 3, dtype=np.int64),
                  np.stack([Q["x"], np.full(nq, -1, np.int32), Q["y"]], 1).reshape(-1))
        qs = range(nq)
        for _ in range(args.warmup):
            pattern_batch_arrays(snap3, *packed)
        ms, nres = [], 0
        barrier_sync()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            r = pattern_batch_arrays(snap3, *packed)
            ms.append(r.ms)
            nres = int(r.offsets[-1])
        barrier_sync()
        dtq = max_over_ranks(time.perf_counter() - t0)
        qps = sum_over_ranks(len(qs) * args.steps) / dtq
        mm = sum(m["ms_match"] for m in ms) / len(ms)
        bm = sum(m["bytes_match"] for m in ms) / len(ms)
        ach = bm / (mm / 1e3) / 1e9 if mm > 0 else 0.0
        pattern = {"metric": "pattern-match queries/sec", "value": round(qps, 1), "unit": "queries/s",
                   "ms_per_step": round(dtq / args.steps * 1e3, 3), "queries_per_step": len(qs),
                   "results_per_step": nres,
                   "workload": "config3: 50M links over 10M nodes, arity 3-6, 64 types, 10K queries",
                   "roofline": {"bound": "hbm", "kernel": "hgx_pattern_match", "achieved": round(ach, 1),
                                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                                "traffic": pmc_traffic("hgx_pattern_match", "config3"),
                                "avg_launch_ms": round(mm, 4), "bytes_per_launch": bm}}
        log(f"rank {rank}: pattern {qps:.1f} q/s, match kernel {mm:.3f} ms")
        snap3.close()
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            pattern["cpu_baseline"] = cpu_query_baseline(g3, Q, args.cpu_budget)
            log(f"cpu pattern baseline {pattern['cpu_baseline']['value']:.1f} q/s")

    # ---------------- config 5: subsumption closures ----------------
    sub = None
    if not args.no_config5:
        sub = run_config5(args, ctx, barrier_sync)

    line = None
    if rank == 0:
        line = {
            "metric": "hyperedge TEPS for batched multi-source BFS; pattern-match queries/sec",
            "value": teps, "unit": "TEPS", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "int32 ids / u64 source bitmasks", "data": "synthetic",
            "config": {"workload": ("config2: 10M nodes / 40M links, Chung-Lu gamma 2.1, arity 2-8, "
                                    f"{args.sources}-source BFS depth {args.depth}") if args.scale == 1.0 else
                       f"config2 at scale {args.scale}, {args.sources} sources, depth {args.depth}",
                       "sources_per_gpu": args.sources, "depth": args.depth, "scale": args.scale,
                       "parallelism": f"sources sharded over {world} rank(s), snapshot replicated"},
            "roofline": roof,
            "cpu_baseline": cpu,
            "device_ms_per_step": round(ms_dev, 3),
            "traversed_edges_per_step": acct["traversed_edges"],
            "union_frontier": acct["union_frontier"],
            "survey_model_bytes_per_step": acct["bytes_survey"],
            "kernels": {k: {"ms_per_step": round(v["ms"] / args.steps, 4), "launches_per_step": v["launches"] / args.steps,
                            "GBps": round(v["bytes"] / (v["ms"] / 1e3) / 1e9, 1) if v["ms"] > 0 else None}
                        for k, v in per_kernel.items()},
            "pattern": pattern,
            "subsumption": sub,
        }

    # ---------------- config 4: 1B incidences, replicated vs hash-partitioned ----------------
    if not args.no_config4:
        import threading
        c4 = {}

        def watchdog():   # a hung collective must not cost the whole line
            log(f"rank {rank}: config4 legs exceeded {args.c4_timeout:.0f}s; reporting what finished")
            if line is not None:
                line["config4"] = dict(c4, error=f"abandoned after {args.c4_timeout:.0f}s")
                emit(line)
            os._exit(0)

        wd = threading.Timer(args.c4_timeout, watchdog)
        wd.daemon = True
        wd.start()
        try:
            run_config4(args, ctx, barrier_sync, c4)
        except Exception as e:   # report, keep the main line
            log(f"rank {rank}: config4 failed: {e!r}")
            c4["error"] = repr(e)
        wd.cancel()
        if line is not None:
            line["config4"] = c4
    if rank == 0:
        emit(line)
    ctx.close()


if __name__ == "__main__":
    main()
