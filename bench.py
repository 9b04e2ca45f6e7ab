#!/usr/bin/env python3
"""Benchmark: hyperedge TEPS of batched multi-source BFS (+ pattern-match queries/sec).

Workload (BASELINE.json configs[1]): config 2 -- 10M nodes, 40M links, arity
U{2..8}, Chung-Lu gamma 2.1, 1024-source BFS to depth 4 on one MI355X.  A step = one
hgx_bfs_batch over the 1024 sources with the CSR resident in HBM (all per-depth visited sets
materialised on the device).  Secondary: config 3, one step = one hgx_pattern_batch of 10,000
hg.and(hg.type(T), hg.incident(a), hg.orderedLink(x, ANY, y)) queries over 50M typed links.

A timed step ends with the result readout: the per-source, per-depth counts of every start atom
(hgx_bfs_result_counts: one counting launch per level over the device rows + one D2H), as
BASELINE.md section 2 times "to the last D2H of results".

Multi-GPU: `python bench.py --gpus N` launches N ranks itself (one process per GPU, RANK /
LOCAL_RANK / WORLD_SIZE / MASTER_* set for each) unless it already runs under
torch.distributed.run, in which case WORLD_SIZE must equal N.  Config 2: the sources are
independent units; every rank holds a replica of the snapshot and runs its own 1024-source batch
(weak scaling, no data-path collective).  Config 4: the same 1024 sources over a partitioned
snapshot (strong scaling, RCCL exchange per level).  torch.distributed (gloo, CPU) carries only
the barrier, the max/sum of scalars and the RCCL unique id.

The CPU baseline is the C restatement of the reference path (oracle/, test infrastructure) timed
on the host cores on a bounded sample of the same workload: 1 thread and all cores (the box's
share), median of 5 runs after 1 warm-up, with the host's core count and CPU model.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def log(msg):
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _git_sha(path):
    try:
        return subprocess.run(["git", "-C", ROOT, "log", "-1", "--format=%h", "--", path], capture_output=True,
                              text=True, timeout=10).stdout.strip() or None
    except Exception:
        return None


def pmc_traffic(kernel, workload):
    """HBM bytes per launch from a committed rocprofv3 PMC summary (profiles/pmc_<workload>.json,
    written by tools/pmc_summary.py with the gfx950 FETCH_SIZE correction) and where it came from:
    (bytes or None, "profiles/pmc_<workload>.json@<commit>").  Counters cannot be collected inside
    this run (rocprofv3 --pmc needs its own pass), so the figure is the committed measurement of the
    same kernel on the same workload, labelled as such."""
    rel = os.path.join("profiles", f"pmc_{workload}.json")
    p = os.path.join(ROOT, rel)
    if not os.path.exists(p):
        return None, None
    try:
        d = json.load(open(p))
        v = d.get("kernels", {}).get(kernel, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None, None
    # the commit the passes measured, written into the file by tools/pmc_summary.py (a GPU lease has
    # no .git); the file's own last commit otherwise
    sha = d.get("commit") or _git_sha(rel)
    return v, f"{rel}@{sha}" if sha else rel


def with_traffic(roof, kernel, workload, avg_launch_ms):
    """The counter-based roofline (VERDICT r4 'do this' 1): `traffic` = the committed PMC HBM bytes per
    launch of `kernel` (profiles/pmc_<workload>.json, named in `traffic_from` as file@commit), `achieved` =
    traffic / this run's average launch time (HIP events), `frac` = achieved / peak.  The implementation's
    algorithmic-byte rate stays beside it as achieved_algorithmic / frac_algorithmic.  Without a committed
    counter pass the algorithmic figure is all there is (frac_from says which)."""
    traffic, src = pmc_traffic(kernel, workload)
    roof["achieved_algorithmic"] = roof.pop("achieved")
    roof["frac_algorithmic"] = roof.pop("frac")
    roof["traffic"], roof["traffic_from"] = traffic, src
    avg_s = avg_launch_ms / 1e3
    if traffic and avg_s > 0:
        ach = traffic / avg_s / 1e9
        roof["achieved"], roof["frac"], roof["frac_from"] = round(ach, 1), round(ach / HBM_PEAK_GBS, 4), "pmc"
        roof["traffic_over_algorithmic"] = round(traffic / roof["bytes_per_launch"], 3) if roof.get("bytes_per_launch") else None
    else:
        roof["achieved"], roof["frac"], roof["frac_from"] = roof["achieved_algorithmic"], roof["frac_algorithmic"], "algorithmic"
    return roof


def roofline(stats_list, workload):
    """Dominant kernel of the BFS step: achieved = PMC HBM bytes per launch / its average launch time
    (HIP events); the algorithmic-byte rate beside it."""
    from hypergraphdb_amd._lib import KERNELS
    tot = {k: {"ms": 0.0, "bytes": 0.0, "launches": 0} for k in KERNELS}
    for st in stats_list:
        for k, v in st["kernels"].items():   # + hgx_bfs_block when the workgroup stage ran
            t = tot.setdefault(k, {"ms": 0.0, "bytes": 0.0, "launches": 0})
            t["ms"] += v["ms"]
            t["bytes"] += v["bytes"]
            t["launches"] += v["launches"]
    dom = max(tot, key=lambda k: tot[k]["ms"])
    t = tot[dom]
    achieved = t["bytes"] / (t["ms"] / 1e3) / 1e9 if t["ms"] > 0 else 0.0
    roof = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "bytes_per_launch": t["bytes"] / max(t["launches"], 1),
            "avg_launch_ms": t["ms"] / max(t["launches"], 1), "launches": t["launches"]}
    return with_traffic(roof, dom, workload, roof["avg_launch_ms"]), tot


def host_info():
    """nproc, the cores this process may use, and the lscpu model name (from /proc/cpuinfo)."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    return {"nproc": os.cpu_count() or 1, "usable_cpus": usable, "cpu_model": model}


def cpu_threads():
    """The CPU share of this job: the GPU box exposes the whole machine to os.cpu_count() (256 CPUs on
    an 8-GPU node) but a one-GPU job owns 16 of them (OMP_NUM_THREADS is set to that share there)."""
    env = os.environ.get("HGX_CPU_THREADS") or os.environ.get("OMP_NUM_THREADS")
    if env:
        return max(1, int(env))
    return max(1, min(16, host_info()["usable_cpus"]))


def median_runs(run, reps=5):
    """run() -> (units, seconds); one warm-up, then the median rate of `reps` runs."""
    run()
    rates = sorted(u / max(sec, 1e-9) for u, sec in (run() for _ in range(reps)))
    return rates[len(rates) // 2], rates


def cpu_leg(run_for_threads, unit, sample, kind="port"):
    """The 1-thread leg and the job's-CPU-share leg (cpu_threads() threads) of one CPU baseline.  `value`
    and `cores` are the share leg as run; `value_linear_usable_cpus` = the 1-thread rate x every CPU the
    process may use, a linear-scaling ceiling for a run on the whole machine (not measured: the box
    gives a one-GPU job 16 CPUs)."""
    info = host_info()
    out = {"unit": unit, "kind": kind, "sample": sample, "repetitions": "median of 5 after 1 warm-up", **info}
    nt = cpu_threads()
    for tag, th in (("1t", 1), (f"{nt}t", nt)):
        med, rates = median_runs(lambda: run_for_threads(th))
        out[f"value_{tag}"] = med
        out[f"rates_{tag}"] = [round(r, 1) for r in rates]
    out["value"] = out[f"value_{nt}t"]
    out["cores"] = nt
    out["cores_note"] = (f"{nt} threads = the CPU share of this job (OMP_NUM_THREADS / HGX_CPU_THREADS, else min(16, "
                         "usable CPUs)); usable_cpus is the whole machine")
    out["value_linear_usable_cpus"] = out["value_1t"] * info["usable_cpus"]
    return out


def cpu_bfs_baseline(g, seeds, depth, budget_s, full_traversals=True):
    """C restatement (oracle/) of HGBreadthFirstTraversal + DefaultALGenerator, one traversal per
    thread, each stopped after budget_s: the edge rate of the reference path over the first budget_s
    of each traversal (a bounded sample of the same workload)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle_ctypes import OracleGraph
    t0 = time.time()
    orc = OracleGraph(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    log(f"cpu baseline: host snapshot built in {time.time() - t0:.1f}s")

    def run(threads):
        batch = np.asarray(seeds[:threads], np.int32)
        tm = {}
        _, tr = orc.bfs_many(batch, depth, depth + 1, nthreads=threads, time_budget_s=budget_s, timing=tm)
        return int(tr.sum()), tm["elapsed_s"]

    out = cpu_leg(run, "TEPS", f"config-2 sources seeds[:threads] (1 thread / the job's CPU share), depth {depth}, one traversal "
                  f"per thread, each stopped after {budget_s:g}s (C restatement of HGBreadthFirstTraversal/"
                  "DefaultALGenerator)")
    # the 2-s prefix of a traversal is its hub-heavy start; a second sample runs one COMPLETE depth-4
    # traversal per thread of the job's share (one run: ~1 min of CPU work)
    if full_traversals:
        nt = cpu_threads()
        tm = {}
        _, tr = orc.bfs_many(np.asarray(seeds[:nt], np.int32), depth, depth + 1, nthreads=nt, timing=tm)
        out["complete_traversals"] = {"threads": nt, "traversals": nt, "seconds": round(tm["elapsed_s"], 2),
                                      "traversed_edges": int(tr.sum()), "value": int(tr.sum()) / tm["elapsed_s"],
                                      "unit": "TEPS", "sample": f"seeds[:{nt}], one complete depth-{depth} traversal per "
                                                                "thread, one run"}
        log(f"cpu baseline: {nt} complete traversals {out['complete_traversals']['value']:.3e} TEPS "
            f"({tm['elapsed_s']:.1f}s)")
    del orc
    return out


def cpu_query_baseline(g, qs, budget_s):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle_ctypes import OracleGraph
    orc = OracleGraph(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])

    # the whole 10K batch in ONE parallel region with dynamic scheduling (og_and_query_many: schedule
    # dynamic, 4), timed to its completion -- per-slice calls each waited for their slowest hub query
    n = len(qs["type"])
    inc_off = np.arange(n + 1, dtype=np.int64)
    pat_off = np.arange(0, 3 * n + 1, 3, dtype=np.int64)
    pat = np.stack([qs["x"], np.full(n, -1, np.int32), qs["y"]], 1).reshape(-1)
    ho = np.ones(n, np.int32)

    def run(threads):
        t1 = time.perf_counter()
        orc.and_query_many(qs["type"], inc_off, qs["a"], pat_off, pat, ho, nthreads=threads)
        return n, time.perf_counter() - t1

    out = cpu_leg(run, "queries/s", f"the {n} config-3 queries as one batch, one OpenMP region with dynamic "
                  "scheduling, to completion (C restatement of AndToQuery + ZigZagIntersectionResult + "
                  "OrderedLinkCondition)")
    del orc
    return out


def _kernel_roof(stats_list, workload=None):
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
    roof = {"bound": "hbm", "kernel": dom, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "avg_launch_ms": round(t["ms"] / max(t["launches"], 1), 4),
            "bytes_per_launch": t["bytes"] / max(t["launches"], 1)}
    return with_traffic(roof, dom, workload, roof["avg_launch_ms"]) if workload else roof


def run_config4(args, ctx, barrier_sync, result):
    """Config 4 (1B incidences) in its two multi-GPU forms:
      replicated  -- every GPU holds the whole snapshot (one-part shard, ~16 GB of CSR) and runs its
                     own 1024-source batch (weak scaling: throughput of the batch workload, no
                     data-path collective);
      partitioned -- the snapshot is split over the N GPUs as a vertex cut (every link on one part,
                     hgx_partition_plan) and the same 1024 sources run together: per level each part
                     expands its own links, then reduce + broadcast of the new rows over RCCL
                     (strong scaling; hgx_pbfs_batch).
    Fills result[...] in place so a watchdog can still report what finished."""
    from hypergraphdb_amd import dist as hdist
    from hypergraphdb_amd import synth
    from hypergraphdb_amd.partition import RcclComm, Shard, ShardSnapshot, partition_plan, pbfs_batch, pbfs_batch_group
    rank, world, local = ctx.rank, ctx.world, ctx.device
    t0 = time.time()
    g = synth.config4(scale=args.c4_scale, n_sources=args.sources)
    log(f"rank {rank}: config4 generated in {time.time() - t0:.1f}s: A={g['num_atoms']} P={len(g['tgt_idx'])}")
    wl = (f"config4: 100M nodes / 200M links (1.0B incidences), Chung-Lu gamma 2.1, {args.sources}-source BFS "
          f"depth {args.depth}" if args.c4_scale == 1.0 else f"config4 at scale {args.c4_scale}")

    last = {}

    def timed(run, n_steps):
        barrier_sync()
        t1 = time.perf_counter()
        st = []
        for _ in range(n_steps):
            r = run()
            last["counts"] = r.counts()   # the readout (the last step's counts are checked below)
            st.append(r.stats(accounting=False, raw=True))
            r.close()
        barrier_sync()
        return ctx.max(time.perf_counter() - t1), [x.as_dict() for x in st]

    # replicated snapshot, one 1024-source batch per GPU
    t0 = time.time()
    sh = Shard.build(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"], 1, 0,
                     np.zeros(len(g["link_atom"]), np.int32))
    snap = ShardSnapshot(sh, local)
    log(f"rank {rank}: config4 replica (one part, {sh.n_local} atoms with incidence) on device in "
        f"{time.time() - t0:.1f}s")
    sh.close()
    snap.set_timing(True)
    mine = hdist.rank_sources(g, args.sources, rank)
    ref_counts = None   # rank 0's replica batch runs g["seeds"]: the partitioned leg's expected counts
    for _ in range(max(args.warmup, 1)):
        r = pbfs_batch_group([snap], mine, args.depth)
        acct = r.parts[0].stats(accounting=True)
        if ref_counts is None:
            ref_counts = r.parts[0].counts()
        r.close()
    ref_edges = acct["traversed_edges"] if rank == 0 else 0.0
    dt, st = timed(lambda: pbfs_batch_group([snap], mine, args.depth).parts[0], args.steps)
    edges = ctx.sum(acct["traversed_edges"] * args.steps)
    result["replicated"] = {
        "metric": "hyperedge TEPS", "value": edges / dt, "unit": "TEPS", "scaling": "weak",
        "ms_per_step": round(dt / args.steps * 1e3, 3), "workload": wl, "n_gpus": world,
        "parallelism": f"snapshot replicated on {world} GPU(s), {args.sources} sources per GPU",
        "traversed_edges_per_step": edges / args.steps, "roofline": _kernel_roof(st, "config4")}
    log(f"rank {rank}: config4 replicated {edges / dt:.3e} TEPS, {dt / args.steps * 1e3:.1f} ms/step")
    snap.close()
    del snap
    if world == 1:
        result["partitioned"] = dict(result["replicated"], scaling="strong",
                                     parallelism="one part: the partition degenerates to the replica",
                                     parity="n/a: one part is the replica")
        return
    # vertex cut over the ranks (every rank computes the same plan), RCCL reduce + broadcast per level
    seeds = g["seeds"]
    t0 = time.time()
    plan = partition_plan(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"], world)
    t_plan = time.time() - t0
    sh = Shard.build(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"], world, rank, plan)
    info = {"local_atoms": sh.n_local, "owned_atoms": sh.n_owned, "local_links": sh.n_links, "local_pins": sh.n_pins,
            "plan_s": round(t_plan, 1)}
    snap = ShardSnapshot(sh, local)
    sh.close()
    del g, plan
    snap.set_timing(True)
    # RCCL between the ranks; HGX_BENCH_C4_TRANSPORT=host stages the exchange through the gloo group
    # (hgx_comm_host_create), which lets a test run the N > 1 leg as two ranks on one GPU
    if os.environ.get("HGX_BENCH_C4_TRANSPORT", "rccl") == "host":
        from hypergraphdb_amd.partition import HostComm
        comm = HostComm.gloo(ctx.dist, world, rank)
    else:
        comm = RcclComm.create(world, rank, local, broadcast=ctx.broadcast_bytes)
    log(f"rank {rank}: config4 part {rank}/{world} on device + {type(comm).__name__} in {time.time() - t0:.1f}s {info}")
    for _ in range(max(args.warmup, 1)):
        r = pbfs_batch(snap, comm, seeds, args.depth)
        acct = r.stats(accounting=True)
        r.close()
    dt, st = timed(lambda: pbfs_batch(snap, comm, seeds, args.depth), args.steps)
    edges_part = ctx.sum(acct["traversed_edges"])
    edges = edges_part * args.steps   # parts' shares sum to the whole batch's numerator
    xbytes = ctx.sum(sum(s["bytes_exchanged"] for s in st)) / args.steps
    xms = ctx.max(sum(s["ms_exchange"] for s in st) / args.steps)
    # self-check, outside the timed region: the parts' per-source per-depth counts of the last timed
    # step, summed over the ranks, must equal the replica's counts of the same sources (rank 0 ran
    # them on the whole snapshot above), and so must the TEPS numerator
    pc = last["counts"]
    width = max(pc.shape[1], ref_counts.shape[1] if rank == 0 else 0)
    width = int(ctx.max(width))
    padded = np.zeros((len(seeds), width), np.int64)
    padded[:, : pc.shape[1]] = pc
    total = ctx.sum_array(padded)
    if os.environ.get("HGX_BENCH_INJECT_MISMATCH") == "1":   # test hook: the check must catch this
        total[0, 1] += 1
    ok = 1.0
    if rank == 0:
        ref = np.zeros((len(seeds), width), np.int64)
        ref[:, : ref_counts.shape[1]] = ref_counts
        ok = float(np.array_equal(total, ref) and edges_part == ref_edges)
    ok = ctx.sum(ok if rank == 0 else 0.0) == 1.0
    log(f"rank {rank}: config4 partitioned parity against the replica: {'ok' if ok else 'MISMATCH'}")
    result["partitioned"] = {
        "metric": "hyperedge TEPS", "value": edges / dt, "unit": "TEPS", "scaling": "strong",
        "ms_per_step": round(dt / args.steps * 1e3, 3), "workload": wl, "n_gpus": world,
        "parallelism": f"vertex cut over {world} GPUs (links placed by hgx_partition_plan), "
                       f"{'RCCL' if isinstance(comm, RcclComm) else 'host-staged gloo'} reduce + broadcast of new "
                       "rows per level, the same sources on every part",
        "exchange_bytes_per_step": xbytes, "exchange_kernels_ms_per_step": round(xms, 3),
        "parity": ok,
        "parity_check": ("the last timed step's per-source per-depth counts summed over the parts == the replica's "
                         "counts of the same sources on the whole snapshot (rank 0), and the summed TEPS numerator == "
                         "the replica's; checked after the timed steps"),
        "rank0_part": info, "roofline": _kernel_roof(st, "config4")}
    if not ok:
        result["error"] = "partitioned counts differ from the replica's"
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
    # the two directions of a step run side by side: hg.subsumed on the snapshot, hg.subsumes on an
    # execution context of it (hgx_graph_context: same device arrays, its own stream and scratch), each
    # driven by its own host thread -- one direction's levels are a few tens of microseconds of
    # latency-bound kernels that leave most of the GPU idle
    views = [snap, snap.context()]
    gens = [DefaultALGenerator(v, AtomTypeCondition(T), None, False, True, rev) for v, rev in zip(views, (False, True))]
    log(f"rank {rank}: config5 ({g['n_nodes']} classes, {len(g['link_atom'])} links) ready in {time.time() - t0:.1f}s")
    from concurrent.futures import ThreadPoolExecutor
    pool = ThreadPoolExecutor(1)

    def direction(k, accounting=False):
        r = H.bfs_batch(views[k], g["seeds"], None, gens[k])
        n = int(r.counts()[:, 1:].sum())   # the result readout: per-class closure sizes per depth (D2H)
        st = r.stats(accounting=accounting, raw=not accounting)   # raw structs: converted after the timed loop
        r.close()
        return n, st

    def step(accounting=False, concurrent=True):
        if not concurrent:
            return [direction(0, accounting), direction(1, accounting)]
        f = pool.submit(direction, 1, accounting)
        a = direction(0, accounting)
        return [a, f.result()]

    trav, closure = 0.0, 0
    for _ in range(max(args.warmup, 1)):
        for n, st in step(accounting=True):
            trav += st["traversed_edges"]
            closure += n
    trav /= max(args.warmup, 1)
    closure //= max(args.warmup, 1)
    # the same step with the directions one after the other (reported next to the timed line, with the
    # push kernels' roofline when they run alone: side by side they share the CUs and each launch lasts
    # longer)
    n5 = max(args.steps, 20)   # a step is ~2 ms: at least 20 of them
    t1 = time.perf_counter()
    seq_sts = []
    for _ in range(n5):
        seq_sts += [st for _, st in step(concurrent=False)]
    seq_ms = (time.perf_counter() - t1) / n5 * 1e3
    seq_sts = [x.as_dict() for x in seq_sts]
    # the timed loop runs without HIP timing events (with both directions on the GPU at once they cost
    # ~0.07 of a ~0.4 ms step, profiles/r04zz_c5_{timing,notiming}.log); the per-kernel times behind
    # `roofline` come from an equal loop with them, reported as ms_per_step_with_timing_events
    for v in views:
        v.set_timing(False)
    barrier_sync()
    t1 = time.perf_counter()
    readout = 0
    for _ in range(n5):
        for n, _st in step():
            readout += n
    barrier_sync()
    dt = ctx.max(time.perf_counter() - t1)
    for v in views:
        v.set_timing(True)
    t2 = time.perf_counter()
    sts = []
    for _ in range(n5):
        for n, st in step():
            sts.append(st)
    dt_ev = ctx.max(time.perf_counter() - t2)
    sts = [x.as_dict() for x in sts]
    drop = None if args.no_dropin else dropin_config5(args, ctx, barrier_sync, g, views, gens, pool)
    pool.shutdown()
    views[1].close()
    assert readout == closure * n5, "config-5 readout differs from the warm-up closures"
    edges = ctx.sum(trav * n5)
    out = {"metric": "hyperedge TEPS (subsumption closures)", "value": edges / dt, "unit": "TEPS",
           "closures_per_s": ctx.sum(2 * len(g["seeds"]) * n5) / dt, "scaling": "weak", "steps": n5,
           "ms_per_step": round(dt / n5 * 1e3, 3), "levels": max(s["n_levels_expanded"] for s in sts),
           "directions": "concurrent: hg.subsumed on the snapshot, hg.subsumes on an execution context of it",
           "ms_per_step_directions_serial": round(seq_ms, 3),
           "ms_per_step_with_timing_events": round(dt_ev / n5 * 1e3, 3),
           "closure_atoms_per_step": closure,
           "workload": (f"config5: {g['n_nodes']} classes, HGSubsumes DAG + noise links, {len(g['seeds'])} classes x "
                        "{subsumed, subsumes}, unbounded depth"),
           "roofline": _kernel_roof(sts, "config5"),
           "roofline_directions_serial": _kernel_roof(seq_sts, "config5")}
    log(f"rank {rank}: config5 {out['value']:.3e} TEPS, {out['closures_per_s']:.1f} closures/s, "
        f"{out['ms_per_step']} ms/step ({seq_ms:.3f} with the directions one after the other), {out['levels']} levels")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        from oracle_ctypes import OracleGraph, algen
        orc = OracleGraph(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])

        def run(threads):
            tm, tr, el = {}, 0, 0.0
            for rev in (False, True):
                _, t_ = orc.bfs_many(g["seeds"], -1, 4096, algen(T, False, True, rev, False), nthreads=threads,
                                     time_budget_s=args.cpu_budget / 2, timing=tm)
                tr += int(t_.sum())
                el += tm["elapsed_s"]
            return tr, el

        out["cpu_baseline"] = cpu_leg(run, "TEPS", f"the {len(g['seeds'])} closures of each direction, every "
                                      f"traversal stopped after {args.cpu_budget / 2:g}s (C restatement of the "
                                      "subsumption BFS)")
        # the whole step on the CPU: every one of the 2 x 1024 closures to completion on the job's threads, one
        # run (the GPU step's exact work; seconds of CPU time)
        nt = cpu_threads()
        tr_all, el_all = 0, 0.0
        for rev in (False, True):
            tm = {}
            _, t_ = orc.bfs_many(g["seeds"], -1, 4096, algen(T, False, True, rev, False), nthreads=nt, timing=tm)
            tr_all += int(t_.sum())
            el_all += tm["elapsed_s"]
        nclos = 2 * len(g["seeds"])
        out["cpu_baseline"]["complete_traversals"] = {
            "threads": nt, "traversals": nclos, "seconds": round(el_all, 3), "traversed_edges": tr_all,
            "value": tr_all / el_all, "unit": "TEPS", "closures_per_s": nclos / el_all,
            "sample": f"all {len(g['seeds'])} closures of each direction to completion (the GPU step's work), one run"}
        log(f"cpu baseline config5: {nclos} complete closures on {nt} threads in {el_all:.2f}s "
            f"({tr_all / el_all:.3e} TEPS, {nclos / el_all:.1f} closures/s)")
        # the drop-in's unit of work on the CPU: one order-exact traversal (the oracle's FIFO
        # HGBreadthFirstTraversal, every pair materialised) at a time on one thread, the same seeds as the
        # GPU's single-seed calls
        n1 = len(drop["single"]["seeds"]) if drop else 0
        for rev, name in ((False, "subsumed"), (True, "subsumes")) if drop else ():
            lat = []
            for sd in drop["single"]["seeds"]:
                t1 = time.perf_counter()
                orc.bfs(int(sd), -1, algen(T, False, True, rev, False))
                lat.append(time.perf_counter() - t1)
            lat.sort()
            drop["single"][name]["cpu_ms_median"] = round(lat[n1 // 2] * 1e3, 4)
            drop["single"][name]["cpu_ms_p90"] = round(lat[int(n1 * 0.9)] * 1e3, 4)
        if drop:
            drop["single"]["cpu"] = ("C restatement of HGBreadthFirstTraversal + DefaultALGenerator (oracle/), one "
                                     "traversal per call on 1 thread, pairs materialised")
            drop["cpu_baseline"] = {"same_as": "subsumption.cpu_baseline",
                                    "note": "the batched sequence step traverses exactly the set step's closures "
                                            "(same seeds, same FIFO traversal); the CPU restatement's rate is that "
                                            "leg's"}
        del orc
    if drop:
        drop["single"]["seeds"] = len(drop["single"]["seeds"])
    out["dropin"] = drop
    snap.close()
    return out


def dropin_config5(args, ctx, barrier_sync, g, views, gens, pool):
    """What the Java drop-ins run for hg.subsumed(G) / hg.subsumes(S) (GpuTraversalToQuery ->
    HGGpuTraversal -> hgx_bfs_sequence, C/query/cond2qry/ToQueryMap.java:282-312,340-370): the
    order-exact FIFO sequence of every closure, pairs and distances into host arrays.  Batched: the
    1024 closures of each direction per step (directions on two execution contexts, as the set step);
    single: one traversal per call, the drop-in's shape (HGGpuTraversal.next() on one start atom)."""
    import hypergraphdb_amd as H
    rank = ctx.rank

    def direction(k):
        r = H.bfs_sequence(views[k], g["seeds"], None, gens[k])   # readout: the result arrays on the host
        return r

    def step():
        f = pool.submit(direction, 1)
        a = direction(0)
        return [a, f.result()]

    ref = step()
    pairs = sum(int(r.offsets[-1]) for r in ref)
    for _ in range(args.warmup):   # the untimed warm-up steps of the command line (buffer pools, tables)
        step()
    n5 = max(args.steps, 10)
    # timed without HIP timing events, as the set step (config5 above); the stage times behind the
    # rooflines come from the loops below, with them
    for v in views:
        v.set_timing(False)
    barrier_sync()
    t1 = time.perf_counter()
    got = []
    t_steps = []
    for _ in range(n5):
        t_s = time.perf_counter()
        got = step()
        t_steps.append(time.perf_counter() - t_s)
    barrier_sync()
    dt = ctx.max(time.perf_counter() - t1)
    for v in views:
        v.set_timing(True)
    t2 = time.perf_counter()
    for _ in range(n5):
        step()
    dt_ev = ctx.max(time.perf_counter() - t2)
    for a, b in zip(got, ref):
        if not (np.array_equal(a.offsets, b.offsets) and np.array_equal(a.atoms, b.atoms) and
                np.array_equal(a.links, b.links)):
            raise RuntimeError("dropin: a timed sequence step differs from the first")
    # roofline of each direction alone (device time by HIP events): the stage with the largest device time
    # a call -- the workgroup-per-seed kernel (hgx_seq_block), the order-exact grid stage (hgx_seq_coop, the
    # big hg.subsumed closures) or the level engine -- with that direction's own counter pass
    # (profiles/pmc_dropin5_<direction>.json: tools/seq_c5.py --direction under tools/profile_cmd.sh)
    roofs = {}
    reps = 5
    for k, name in ((0, "subsumed"), (1, "subsumes")):
        acc = {"hgx_seq_block": [0.0, 0.0], "hgx_seq_coop": [0.0, 0.0], "level engine": [0.0, 0.0]}
        ms_call = 0.0
        for _ in range(reps):
            r = direction(k)
            acc["hgx_seq_block"][0] += r.ms_block
            acc["hgx_seq_block"][1] += r.bytes_block
            acc["hgx_seq_coop"][0] += r.ms_coop
            acc["hgx_seq_coop"][1] += r.bytes_coop
            # (the reruns' device time brackets the grid stage when it took them: the level engine's own is the rest)
            acc["level engine"][0] += max(0.0, r.ms_level - r.ms_coop) if r.n_coop else r.ms_level
            acc["level engine"][1] += r.bytes_level
            ms_call += r.ms_total
        dom = max(acc, key=lambda x: acc[x][0])
        ms, by = acc[dom][0] / reps, acc[dom][1] / reps
        ach = by / (ms / 1e3) / 1e9 if ms > 0 else 0.0
        roofs[name] = with_traffic({"bound": "hbm", "kernel": dom, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                                    "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 5), "avg_launch_ms": round(ms, 4),
                                    "bytes_per_launch": by, "launches_per_call": 1,
                                    "stages_per_call": {x: {"device_ms": round(v[0] / reps, 4), "algorithmic_bytes": v[1] / reps}
                                                        for x, v in acc.items()},
                                    "seeds_workgroup_engine": r.n_block, "seeds_grid_stage": r.n_coop,
                                    "seeds_level_engine": r.n_level, "ms_per_call": round(ms_call / reps, 4)},
                                   dom, f"dropin5_{name}", ms)
    # single-seed calls: the first 200 classes, one traversal per call, each direction
    single = {"seeds": [int(x) for x in g["seeds"][:200]]}
    for k, name in ((0, "subsumed"), (1, "subsumes")):
        lat = []
        for sd in single["seeds"]:
            t1 = time.perf_counter()
            H.bfs_sequence(views[k], [sd], None, gens[k])
            lat.append(time.perf_counter() - t1)
        lat.sort()
        n1 = len(lat)
        single[name] = {"ms_median": round(lat[n1 // 2] * 1e3, 4), "ms_p90": round(lat[int(n1 * 0.9)] * 1e3, 4),
                        "ms_max": round(lat[-1] * 1e3, 4)}
    out = {"metric": "order-exact closures/s (hgx_bfs_sequence: the HGTraversal drop-in)",
           "value": ctx.sum(2 * len(g["seeds"]) * n5) / dt, "unit": "closures/s", "steps": n5,
           "ms_per_step": round(dt / n5 * 1e3, 3), "ms_per_step_with_timing_events": round(dt_ev / n5 * 1e3, 3),
           # the step time's spread (value and ms_per_step are the whole loop's mean; a few steps take
           # several times the median, tools/seq_c5.py --concurrent shows the same)
           "ms_step_median": round(float(np.median(t_steps)) * 1e3, 3), "ms_step_max": round(max(t_steps) * 1e3, 3),
           "pairs_per_step": pairs, "traversed_items_per_step": sum(r.traversed_edges for r in ref),
           "step": "hgx_bfs_sequence of the 1024 classes per direction, the directions on two execution contexts; "
                   "every (link, atom, distance) pair in host arrays",
           # the step's bound: the direction whose dominant stage takes longer (the directions run side by side)
           "roofline": dict(max(roofs.values(), key=lambda x: x["avg_launch_ms"]),
                            direction=max(roofs, key=lambda n: roofs[n]["avg_launch_ms"])),
           "roofline_subsumed": roofs["subsumed"], "roofline_subsumes": roofs["subsumes"], "single": single}
    log(f"rank {rank}: dropin config5 {out['value']:.1f} closures/s, {out['ms_per_step']} ms/step; single-seed "
        f"subsumed {single['subsumed']['ms_median']} ms, subsumes {single['subsumes']['ms_median']} ms (median)")
    return out


def dropin_config2(args, ctx, snap, g):
    """The order-exact sequence engine on config 2: 64 of the bench's sources to depth 2 in one
    hgx_bfs_sequence call (each traversal returns ~4.5M pairs, so the workgroup engine hands them all
    to the level-synchronous one), pairs into host arrays.  TEPS = traversed incidence items / time."""
    import hypergraphdb_amd as H
    seeds = np.asarray(g["seeds"][:64], np.int32)
    r = H.bfs_sequence(snap, seeds, 2)
    pairs, trav = int(r.offsets[-1]), r.traversed_edges
    del r
    steps = 3
    t1 = time.perf_counter()
    ms_dev = ms_lev = by_lev = 0.0
    pulls = 0
    walls = []
    kept = []   # the callers' arrays live past the timed loop: freeing 3 GB of host arrays (~0.14 s of munmap
    for _ in range(steps):   # a step, measured) is the caller's business, not the traversal's
        tw = time.perf_counter()
        r = H.bfs_sequence(snap, seeds, 2)
        walls.append(round((time.perf_counter() - tw) * 1e3, 1))
        ms_dev += r.ms_total
        ms_lev += r.ms_level
        by_lev += r.bytes_level
        pulls = r.pull_levels
        if int(r.offsets[-1]) != pairs:
            raise RuntimeError("dropin config2: a timed step differs from the first")
        kept.append(r)
    dt = time.perf_counter() - t1
    del kept, r
    # the level engine's roofline over its device time a call (which includes the D2H copy of the pairs): `traffic`
    # = the PMC HBM bytes of every kernel of one steady call summed (profiles/pmc_dropin2.json: tools/seq_c2.py's
    # last call under tools/profile_cmd.sh, --from-last hgx_ls_seed), `frac` = that over this run's device time;
    # the engine's own algorithmic byte count (device counters, hgx_seq_result_level_stats) beside it
    ms_call = ms_lev / steps
    ach_alg = by_lev / steps / (ms_call / 1e3) / 1e9 if ms_call > 0 else 0.0
    roof = {"bound": "hbm", "kernel": "level engine (hgx_ls_* / hgx_lp_* / hgx_lr_*, one call)", "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "ms_per_call": round(ms_call, 3), "algorithmic_bytes_per_call": by_lev / steps,
            "achieved_algorithmic": round(ach_alg, 1), "frac_algorithmic": round(ach_alg / HBM_PEAK_GBS, 4),
            "achieved": round(ach_alg, 1), "frac": round(ach_alg / HBM_PEAK_GBS, 4), "frac_from": "algorithmic",
            "traffic": None, "traffic_from": None,
            "scope": "one hgx_bfs_sequence call: bytes over the level engine's device time, which includes the D2H copy "
                     "of the pairs"}
    rel = os.path.join("profiles", "pmc_dropin2.json")
    if os.path.exists(os.path.join(ROOT, rel)):
        pj = json.load(open(os.path.join(ROOT, rel)))
        ks = pj.get("kernels", {})
        call = sum((v.get("hbm_bytes_per_launch") or 0.0) * v["launches"] for v in ks.values())
        if call > 0 and ms_call > 0:
            a_ = call / (ms_call / 1e3) / 1e9
            roof.update(traffic=call, traffic_from=f"{rel}@{pj.get('commit') or _git_sha(rel)}", achieved=round(a_, 1),
                        frac=round(a_ / HBM_PEAK_GBS, 4), frac_from="pmc",
                        traffic_over_algorithmic=round(call / (by_lev / steps), 3) if by_lev else None,
                        traffic_scope="PMC HBM bytes of every kernel of one steady call, summed")
        hk = {k: v for k, v in ks.items() if k.startswith(("hgx_ls_", "hgx_lp_", "hgx_lr_")) and v.get("hbm_bytes_per_launch")}
        dom = max(hk, key=lambda k: hk[k]["avg_ms"] * hk[k]["launches"], default=None)
        if dom:
            kk = hk[dom]
            a_ = kk["hbm_bytes_per_launch"] / (kk["avg_ms"] / 1e3) / 1e9
            roof["dominant_kernel_pmc"] = {"kernel": dom, "traffic": kk["hbm_bytes_per_launch"],
                                           "avg_launch_ms": kk["avg_ms"], "launches": kk["launches"],
                                           "achieved": round(a_, 1), "frac": round(a_ / HBM_PEAK_GBS, 4)}
    out = {"metric": "hyperedge TEPS of the order-exact sequence", "value": ctx.sum(trav * steps) / ctx.max(dt),
           "unit": "TEPS", "seeds": len(seeds), "depth": 2, "steps": steps, "ms_per_step": round(dt / steps * 1e3, 2),
           "device_ms_per_step": round(ms_dev / steps, 2), "level_engine_ms_per_step": round(ms_lev / steps, 2),
           "pull_levels": pulls, "pairs_per_step": pairs, "traversed_items_per_step": trav, "roofline": roof}
    log(f"rank {ctx.rank}: dropin config2 {out['value']:.3e} TEPS, {out['ms_per_step']} ms/step, {pairs} pairs; "
        f"calls {walls} ms wall (device {out['device_ms_per_step']} ms)")
    if ctx.rank == 0 and ctx.world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        from oracle_ctypes import OracleGraph
        orc = OracleGraph(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])

        def run(threads):
            tm = {}
            _, tr = orc.bfs_many(seeds[: max(threads, 4)], 2, 3, nthreads=threads, time_budget_s=args.cpu_budget,
                                 timing=tm)
            return int(tr.sum()), tm["elapsed_s"]

        out["cpu_baseline"] = cpu_leg(run, "TEPS", f"the first max(threads, 4) of the 64 seeds to depth 2, each "
                                      f"traversal stopped after {args.cpu_budget:g}s (C restatement)")
        del orc
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


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(argv):
    """`bench.py --gpus N` outside torch.distributed.run: start N ranks of this script (one process
    per GPU) and exit with the first failing rank's status.  Runs before anything touches a GPU.
    Under torch.distributed.run (WORLD_SIZE set) nothing is launched, but WORLD_SIZE must equal N."""
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("--gpus", type=int, default=1)
    a, _ = pre.parse_known_args(argv)
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != a.gpus:
            print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={ws}", file=sys.stderr)
            sys.exit(2)
        return
    if a.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr)
        sys.exit(2)
    if a.gpus == 1:
        return
    port = str(_free_port())
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus), LOCAL_WORLD_SIZE=str(a.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        # rank 0 prints the JSON line on our stdout; the other ranks' stdout goes to stderr
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                      stdout=None if r == 0 else sys.stderr.fileno()))
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            c = p.poll()
            if c is None:
                continue
            pending.remove(p)
            if c != 0 and rc == 0:
                rc = c
                for q in pending:   # a failed rank would leave the others waiting in a collective
                    q.terminate()
        time.sleep(0.2)
    sys.exit(rc)


def dry_run(args):
    """CPU-side rehearsal of the launch: every rank joins the gloo group and reports; no GPU work."""
    from hypergraphdb_amd import dist as hdist
    ctx = hdist.init_from_env("gloo")
    ranks = ctx.sum(1.0)
    ctx.barrier()
    if ctx.rank == 0:
        emit({"dry_run": True, "n_gpus": ctx.world, "ranks_joined": int(ranks), "gpus_flag": args.gpus})
    ctx.close()


def main():
    if os.environ.get("HGX_LIB_VARIANT"):   # the bench line measures the product library, never an A/B variant
        raise SystemExit("bench.py: HGX_LIB_VARIANT is set; unset it (A/B variants are for tools/ only)")
    launch_ranks(sys.argv[1:])
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
    ap.add_argument("--cpu-budget", type=float, default=2.0, help="seconds of CPU-baseline work per run")
    ap.add_argument("--no-config4", action="store_true", help="skip the config-4 (1B incidences) legs")
    ap.add_argument("--no-config5", action="store_true", help="skip the config-5 subsumption leg")
    ap.add_argument("--no-dropin", action="store_true", help="skip the order-exact sequence (drop-in) legs")
    ap.add_argument("--c5-scale", type=float, default=1.0, help="fraction of the config-5 size")
    ap.add_argument("--c4-scale", type=float, default=1.0, help="fraction of the config-4 size")
    ap.add_argument("--c4-timeout", type=float, default=420.0,
                    help="seconds after which the config-4 legs are abandoned (the line is still printed)")
    ap.add_argument("--dry-run", action="store_true", help="launch the ranks and join the group only (no GPU)")
    args = ap.parse_args()
    if args.dry_run:
        dry_run(args)
        return

    # a progress line every 30 s on stderr: the CPU-baseline legs run minutes inside one C call (16
    # complete config-2 traversals: ~70-110 s) and a silent run of 3 minutes is taken for a hung one
    import threading
    t_start = time.time()

    def heartbeat():
        while True:
            time.sleep(30)
            log(f"still running ({time.time() - t_start:.0f} s)")

    threading.Thread(target=heartbeat, daemon=True).start()

    from hypergraphdb_amd import dist as hdist
    from hypergraphdb_amd._lib import device_count, device_synchronize

    # one process per GPU; only the barrier and scalar max/sum cross processes (gloo, CPU)
    ctx = hdist.init_from_env("gloo")
    rank, world, local = ctx.rank, ctx.world, ctx.device
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the group has {world} ranks")
    ndev = device_count()
    if local >= ndev:
        raise SystemExit(f"bench.py: rank {rank} needs device {local} but {ndev} HIP device(s) are visible")

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
            acct_visits = int(res.counts().sum())
            log(f"rank {rank}: levels |U_d|={acct['union_frontier']} traversed={acct['traversed_edges']:.3e}")
        res.close()
        log(f"rank {rank}: warmup {w} done")
    if acct is None:
        res = H.bfs_batch(snap, g["seeds"], args.depth)
        acct = res.stats(accounting=True)
        acct_visits = int(res.counts().sum())
        res.close()
    stats = []
    barrier_sync()
    t0 = time.perf_counter()
    readout = 0
    phase = {"bfs_batch": 0.0, "readout": 0.0, "stats+close": 0.0}   # host wall split of the steps
    for _ in range(args.steps):
        ta = time.perf_counter()
        res = H.bfs_batch(snap, g["seeds"], args.depth)
        tb = time.perf_counter()
        readout += int(res.counts().sum())   # the result readout: per-source per-depth counts (D2H)
        tc = time.perf_counter()
        stats.append(res.stats(accounting=False, raw=True))
        res.close()
        phase["bfs_batch"] += tb - ta
        phase["readout"] += tc - tb
        phase["stats+close"] += time.perf_counter() - tc
    barrier_sync()
    log(f"rank {rank}: host wall per step (ms): " +
        ", ".join(f"{k} {v / max(args.steps, 1) * 1e3:.3f}" for k, v in phase.items()))
    dt = max_over_ranks(time.perf_counter() - t0)
    stats = [x.as_dict() for x in stats]
    assert readout == args.steps * acct_visits, "readout differs from the warm-up batch"
    edges_total = sum_over_ranks(acct["traversed_edges"] * args.steps)
    teps = edges_total / dt
    roof, per_kernel = roofline(stats, "config2")
    ms_dev = sum(s["ms_total"] for s in stats) / len(stats)
    # step-level efficiency against the minimum-bytes model: every byte the
    # traversal must move at least once, over the device time of the whole step
    ach_min = acct["bytes_min"] / (ms_dev / 1e3) / 1e9 if ms_dev > 0 else 0.0
    roof["min_bytes"] = {"model": "per level: CSR columns once (or the frontier's CSR slices) + one S/8-byte row "
                                  "per frontier atom read and per new atom written; whole step, device time",
                         "bytes_per_step": acct["bytes_min"], "achieved": round(ach_min, 1),
                         "frac": round(ach_min / HBM_PEAK_GBS, 4)}
    log(f"rank {rank}: {args.steps} steps in {dt:.3f}s -> {teps:.3e} TEPS; device ms/step {ms_dev:.2f}; "
        f"dominant {roof['kernel']} {roof['achieved']} GB/s")
    drop2 = None if args.no_dropin else dropin_config2(args, ctx, snap, g)
    snap.close()
    del snap

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_bfs_baseline(g, g["seeds"], args.depth, args.cpu_budget)
        log(f"cpu baseline {cpu['value_1t']:.3e} TEPS on 1 thread, {cpu['value']:.3e} on {cpu['cores']} threads")
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
        from hypergraphdb_amd.query import QuerySet, pattern_batch_arrays
        nq = len(Q["type"])
        # hg.and(hg.type(T), hg.incident(a), hg.orderedLink(x, hg.anyHandle(), y)) as one packed batch
        packed = (Q["type"], np.arange(nq + 1, dtype=np.int64), Q["a"], np.ones(nq, np.int32),
                  np.arange(0, 3 * nq + 1, 3, dtype=np.int64),
                  np.stack([Q["x"], np.full(nq, -1, np.int32), Q["y"]], 1).reshape(-1))
        qs = range(nq)
        # the step: the 10K queries resident in HBM (hgx_query_set_create, outside the timed region, as
        # the contract has every input resident), one hgx_pattern_batch_set_into, the result readout
        # (offsets and ids, written by the kernels into mapped host memory, copied into the caller's
        # arrays); the arrays are sized from a warm-up run and a step that outgrows them fails
        qset = QuerySet(snap3, *packed)
        r0 = qset.run(snap3)
        q_off = np.zeros(nq + 1, np.int64)
        q_ids = np.zeros(max(1, int(r0.offsets[-1])), np.int32)
        # a step is ~0.07 ms: at least 50 of them, so the timer and the barriers are not a share of it.
        # The timed steps run without the HIP timing events (four event records and an elapsed-time
        # query per batch are instrumentation, ~13 us of host time a step); the match kernel's launch
        # time for the roofline comes from the same number of steps run with timing on, after.
        n3 = max(args.steps, 50)
        tim = np.zeros((n3, 3), np.float64)
        snap3.set_timing(False)
        for _ in range(max(args.warmup, 3)):
            qset.run_into(snap3, q_off, q_ids)
        nres = 0
        barrier_sync()
        t0 = time.perf_counter()
        for i in range(n3):
            nres = qset.run_into(snap3, q_off, q_ids)
        barrier_sync()
        dtq = max_over_ranks(time.perf_counter() - t0)
        if nres > len(q_ids) or not np.array_equal(q_off, r0.offsets) or not np.array_equal(q_ids[:nres], r0.ids):
            raise RuntimeError("config3: the timed batches differ from the first run")
        snap3.set_timing(True)
        t1 = time.perf_counter()
        for i in range(n3):
            qset.run_into(snap3, q_off, q_ids, tim[i])
        ms_timed = (time.perf_counter() - t1) / n3 * 1e3
        ms = [{"ms_total": t[0], "ms_match": t[1], "bytes_match": t[2]} for t in tim]
        qps = sum_over_ranks(len(qs) * n3) / dtq
        qset.close()
        # the same batch handed over in host memory each step (hgx_pattern_batch_packed: the queries
        # cross PCIe inside the step) -- the PCIe-inclusive rate, reported beside the line
        for _ in range(args.warmup):
            pattern_batch_arrays(snap3, *packed)
        t1 = time.perf_counter()
        for _ in range(n3):
            pattern_batch_arrays(snap3, *packed)
        dtp = time.perf_counter() - t1
        mm = sum(m["ms_match"] for m in ms) / len(ms)
        bm = sum(m["bytes_match"] for m in ms) / len(ms)
        ach = bm / (mm / 1e3) / 1e9 if mm > 0 else 0.0
        pattern = {"metric": "pattern-match queries/sec", "value": round(qps, 1), "unit": "queries/s",
                   "ms_per_step": round(dtq / n3 * 1e3, 3), "steps": n3, "queries_per_step": len(qs),
                   "results_per_step": nres,
                   "ms_per_step_with_timing_events": round(ms_timed, 3),
                   "device_ms_per_batch": round(sum(t[0] for t in tim) / len(tim), 4),
                   "inputs": "the 10K packed queries resident in HBM (hgx_query_set_create before the timed steps)",
                   "results": "offsets + ids into preallocated host arrays each step (hgx_pattern_batch_set_into)",
                   "pcie_inclusive": {"value": round(len(qs) * n3 / dtp, 1), "unit": "queries/s",
                                      "ms_per_step": round(dtp / n3 * 1e3, 3),
                                      "path": "hgx_pattern_batch_packed: host arrays staged and read over PCIe each step"},
                   "workload": "config3: 50M links over 10M nodes, arity 3-6, 64 types, 10K queries",
                   "roofline": with_traffic({"bound": "hbm", "kernel": "hgx_pattern_match_flat",
                                             "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                             "frac": round(ach / HBM_PEAK_GBS, 4), "avg_launch_ms": round(mm, 4),
                                             "bytes_per_launch": bm}, "hgx_pattern_match_flat", "config3", mm)}
        log(f"rank {rank}: pattern {qps:.1f} q/s ({len(qs) * n3 / dtp:.1f} with the queries crossing PCIe each "
            f"step), match kernel {mm:.3f} ms")
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
            "dropin": None if args.no_dropin else {
                "what": "hgx_bfs_sequence, the order-exact FIFO next() sequence the Java drop-ins run "
                        "(HGGpuTraversal; hg.subsumed / hg.subsumes through GpuTraversalToQuery)",
                "config5": sub.pop("dropin") if sub else None, "config2": drop2},
        }

    # ---------------- config 4: 1B incidences, replicated vs hash-partitioned ----------------
    rc = 0
    if not args.no_config4:
        import threading
        c4 = {}

        def watchdog():   # a hung collective must not cost the whole line, but the run has failed
            log(f"rank {rank}: config4 legs exceeded {args.c4_timeout:.0f}s; reporting what finished")
            if line is not None:
                line["config4"] = dict(c4, error=f"abandoned after {args.c4_timeout:.0f}s")
                emit(line)
            os._exit(3)

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
        if "error" in c4:   # a failed or mismatching config-4 leg fails the run (after the line is out)
            rc = 3
    if rank == 0:
        emit(line)
    ctx.close()
    if rc:
        sys.exit(rc)


if __name__ == "__main__":
    main()
