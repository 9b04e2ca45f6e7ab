#!/usr/bin/env python3
"""Partitioned-BFS rehearsal on ONE GPU: config 4 (scaled) split into NP in-process parts on cuda:0.

The parts share the device, so wall time is the aggregate work of all parts, not a multi-GPU
time; what this measures is what one GPU of an NP-GPU run would carry: its local atoms / links /
pins, its kernels' device time and the ghost-row bytes it ships per level.

  python tools/bench_part.py --scale 0.25 --parts 1 2 4 8 --out gpurun_out/part.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=0.25)
    ap.add_argument("--parts", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--sources", type=int, default=1024)
    ap.add_argument("--depth", type=int, default=4)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    from hypergraphdb_amd import synth
    from hypergraphdb_amd.partition import Shard, ShardSnapshot, pbfs_batch_group
    t0 = time.time()
    g = synth.config4(scale=args.scale, n_sources=args.sources)
    print(f"config4 x{args.scale}: A={g['num_atoms']} P={len(g['tgt_idx'])} in {time.time() - t0:.1f}s", flush=True)
    rows = []
    ref_counts = None
    for NP in args.parts:
        t0 = time.time()
        snaps, info = [], []
        for p in range(NP):
            sh = Shard.build(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"], NP, p)
            info.append({"local_atoms": sh.n_local, "local_links": sh.n_links, "local_pins": sh.n_pins})
            snaps.append(ShardSnapshot(sh, 0))
            sh.close()
            snaps[-1].set_timing(True)
        build_s = time.time() - t0
        r = pbfs_batch_group(snaps, g["seeds"], args.depth)
        counts = r.counts()
        st0 = r.stats(accounting=True)
        r.close()
        if ref_counts is None:
            ref_counts = counts
        assert np.array_equal(counts, ref_counts), f"{NP} parts differ from {args.parts[0]}"
        t0 = time.perf_counter()
        sts = []
        for _ in range(args.steps):
            r = pbfs_batch_group(snaps, g["seeds"], args.depth)
            sts.append(r.stats(accounting=False))
            r.close()
        wall = (time.perf_counter() - t0) / args.steps
        per = []
        for p in range(NP):
            ss = [s[p] for s in sts]
            per.append({"device_ms": sum(s["ms_total"] for s in ss) / len(ss),
                        "kernel_ms": {k: round(sum(s["kernels"][k]["ms"] for s in ss) / len(ss), 3)
                                      for k in ss[0]["kernels"]},
                        "exchange_ms": sum(s["ms_exchange"] for s in ss) / len(ss),
                        "bytes_exchanged": sum(s["bytes_exchanged"] for s in ss) / len(ss),
                        "traversed_edges": st0[p]["traversed_edges"], **info[p]})
        row = {"parts": NP, "build_s": round(build_s, 1), "wall_ms_all_parts": round(wall * 1e3, 2),
               "traversed_edges": sum(x["traversed_edges"] for x in per),
               "max_part_kernel_ms": round(max(sum(x["kernel_ms"].values()) for x in per), 3),
               "max_part_exchange_ms": round(max(x["exchange_ms"] for x in per), 3),
               "exchange_bytes_total": sum(x["bytes_exchanged"] for x in per), "per_part": per}
        rows.append(row)
        print(json.dumps({k: v for k, v in row.items() if k != "per_part"}), flush=True)
        for s in snaps:
            s.close()
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"scale": args.scale, "sources": args.sources, "depth": args.depth, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
