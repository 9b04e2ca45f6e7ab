#!/usr/bin/env python3
"""Config 4 on one GPU with S = 128..1024 sources (the per-GPU share of the replicated,
source-split strong-scaling variant at 8..1 GPUs).

  python tools/bench_c4_sources.py --scale 1.0 --sizes 128 256 512 1024
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--sizes", type=int, nargs="+", default=[128, 256, 512, 1024])
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    from hypergraphdb_amd import synth
    from hypergraphdb_amd.partition import Shard, ShardSnapshot, pbfs_batch_group
    g = synth.config4(scale=args.scale)
    sh = Shard.build(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"], 1, 0)
    snap = ShardSnapshot(sh, 0)
    sh.close()
    snap.set_timing(True)
    rows = []
    for S in args.sizes:
        seeds = g["seeds"][:S]
        r = pbfs_batch_group([snap], seeds, 4)
        acct = r.parts[0].stats(accounting=True)
        r.close()
        t0 = time.perf_counter()
        ms = []
        for _ in range(args.steps):
            r = pbfs_batch_group([snap], seeds, 4)
            st = r.parts[0].stats(accounting=False)
            ms.append({k: v["ms"] for k, v in st["kernels"].items()})
            r.close()
        dt = (time.perf_counter() - t0) / args.steps
        row = {"sources": S, "ms_per_step": round(dt * 1e3, 2), "teps": acct["traversed_edges"] / dt,
               "kernel_ms": {k: round(sum(m[k] for m in ms) / len(ms), 2) for k in ms[0]}}
        rows.append(row)
        print(json.dumps(row), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"scale": args.scale, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
