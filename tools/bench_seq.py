#!/usr/bin/env python3
"""Order-exact traversal (hgx_bfs_sequence) throughput on config 2: hyperedge TEPS of the FIFO
next() sequence for a batch of seeds, checked against the C restatement for a sample of seeds.

  python tools/bench_seq.py [--scale 1.0] [--seeds 64] [--depth 4] [--check 4]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--seeds", type=int, default=64)
    ap.add_argument("--depth", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--check", type=int, default=4, help="seeds compared with the oracle")
    args = ap.parse_args()
    import hypergraphdb_amd as H
    from hypergraphdb_amd import synth
    g = synth.config2(scale=args.scale, n_sources=max(args.seeds, 1))
    seeds = g["seeds"][: args.seeds]
    snap = H.HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    snap.set_timing(True)
    out = {"workload": f"config2 scale {args.scale}", "seeds": len(seeds), "depth": args.depth, "runs": []}
    res = None
    for r in range(args.rounds + 1):
        t0 = time.perf_counter()
        res = H.bfs_sequence(snap, seeds, args.depth)
        dt = time.perf_counter() - t0
        if r:
            out["runs"].append({"wall_s": dt, "device_ms": res.ms_total})
    dev = sorted(x["device_ms"] for x in out["runs"])[len(out["runs"]) // 2]
    wall = sorted(x["wall_s"] for x in out["runs"])[len(out["runs"]) // 2]
    out.update(pairs=int(res.offsets[-1]), traversed_edges=res.traversed_edges, device_ms=dev, wall_s=wall,
               teps_device=res.traversed_edges / (dev / 1e3) if dev > 0 else None,
               teps_wall=res.traversed_edges / wall)
    if args.check:
        from oracle_ctypes import OracleGraph
        orc = OracleGraph(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
        ok = 0
        t0 = time.perf_counter()
        for i in range(min(args.check, len(seeds))):
            l, a, d, _ = orc.bfs(int(seeds[i]), args.depth)
            gl, ga, gd = res.pairs(i)
            assert np.array_equal(ga, a) and np.array_equal(gl, l) and np.array_equal(gd, d), i
            ok += 1
        out["oracle_checked_seeds"] = ok
        out["oracle_s_per_seed"] = (time.perf_counter() - t0) / max(ok, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
