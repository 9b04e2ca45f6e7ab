#!/usr/bin/env python3
"""Config-5 closure step split by seed size: where the set engine's time goes.

Times hgx_bfs_batch per direction on (a) all seeds, (b) the seeds whose closure exceeds --big
pairs, (c) the rest, and prints the closure-size distribution (from the batch's own counts).

  python tools/c5_split.py [--big 2046] [--reps 10]
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
    ap.add_argument("--big", type=int, default=2046)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import hypergraphdb_amd as H
    from hypergraphdb_amd import AtomTypeCondition, DefaultALGenerator, synth
    g = synth.config5()
    snap = H.HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    T = g["subsumes_type"]
    rep = {}
    for rev, name in ((False, "subsumed"), (True, "subsumes")):
        gen = DefaultALGenerator(snap, AtomTypeCondition(T), None, False, True, rev)
        r = H.bfs_batch(snap, g["seeds"], None, gen)
        c = r.counts()
        r.close()
        size = c[:, 1:].sum(1)
        depth = np.array([int(np.nonzero(x)[0].max()) for x in c])
        big = np.nonzero(size > args.big)[0]
        small = np.nonzero(size <= args.big)[0]
        d = {"sizes": {"sum": int(size.sum()), "max": int(size.max()), "p50": float(np.median(size)),
                       "n_big": int(len(big)), "big_sizes": sorted(size[big].tolist())},
             "depth_max": int(depth.max()), "depth_p50": float(np.median(depth))}
        from hypergraphdb_amd import _lib
        snap.set_timing(True)
        for blk in (1, 0):
            snap.set_option(_lib.HGX_OPT_BFS_BLOCK, blk)
            for part, idx in (("all", np.arange(len(size))), ("big", big), ("small", small)):
                if len(idx) == 0:
                    continue
                sd = np.ascontiguousarray(g["seeds"][idx])
                ts = []
                for _ in range(args.reps):
                    t0 = time.perf_counter()
                    r = H.bfs_batch(snap, sd, None, gen)
                    r.counts()
                    st = r.stats(accounting=False)
                    r.close()
                    ts.append((time.perf_counter() - t0) * 1e3)
                d[f"{part}_block{blk}"] = {
                    "seeds": int(len(idx)), "wall_ms_median": round(float(np.median(ts)), 3),
                    "wall_ms_min": round(float(np.min(ts)), 3), "levels": int(st["n_levels_expanded"]),
                    "device_ms": round(st["ms_total"], 3), "block_seeds": st["block_seeds"],
                    "block_rerun": st["block_rerun"],
                    "block_ms": round(st["kernels"].get("hgx_bfs_block", {}).get("ms", 0.0), 3)}
        rep[name] = d
        print(name, json.dumps(d), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(rep, f, indent=1)
    snap.close()


if __name__ == "__main__":
    main()
