#!/usr/bin/env python3
"""Interleaved A/B of BFS engine options in one process (cdna_hip_programming.md rule 24).

  python tools/ab_bfs.py --flags 0,2,4,6,7 --rounds 3 [--scale 1.0]

For every flag setting (HGX_OPT_BFS_FLAGS) the same config-2 batch runs `rounds` times, interleaved;
prints per-level device ms per kernel and checks that every variant yields identical results: the
per-source per-depth counts of every seed and the visited sets of a sample of seeds.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--flags", default="0,2,4,6,7")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--sources", type=int, default=1024)
    ap.add_argument("--depth", type=int, default=4)
    args = ap.parse_args()
    import hypergraphdb_amd as H
    from hypergraphdb_amd import _lib, synth
    g = synth.config2(scale=args.scale, n_sources=args.sources)
    snap = H.HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    snap.set_timing(True)
    flags = [int(f, 0) for f in args.flags.split(",")]
    res = {f: [] for f in flags}
    ref_new = ref_counts = ref_sets = None
    sample = list(range(0, args.sources, max(1, args.sources // 8)))
    for r in range(args.rounds + 1):
        for f in flags:
            snap.set_option(_lib.HGX_OPT_BFS_FLAGS, f)
            out = H.bfs_batch(snap, g["seeds"], args.depth)
            st = out.stats(accounting=False)
            if r == 0:   # identical results: counts of every seed, sets of the sampled seeds
                counts = out.counts()
                sets = [out.visited(i, d).tobytes() for i in sample for d in range(counts.shape[1])]
                if ref_counts is None:
                    ref_counts, ref_sets = counts, sets
                assert counts.shape == ref_counts.shape and (counts == ref_counts).all(), (f, "per-source counts")
                assert sets == ref_sets, (f, "visited sets")
            out.close()
            if ref_new is None:
                ref_new = st["level_new"]
            assert st["level_new"] == ref_new, (f, st["level_new"], ref_new)   # identical frontiers
            if r > 0:   # round 0 = warm-up
                res[f].append(st)
    table = {}
    for f in flags:
        runs = res[f]
        tot = sorted(s["ms_total"] for s in runs)
        k = {name: sorted(s["kernels"][name]["ms"] for s in runs)[len(runs) // 2] for name in runs[0]["kernels"]}
        lv = [round(sorted(s["level_ms"][d] for s in runs)[len(runs) // 2], 3) for d in range(len(runs[0]["level_ms"]))]
        lgbs = [round(runs[0]["level_bytes"][d] / (lv[d] / 1e3) / 1e9, 0) if lv[d] > 0 else None for d in range(len(lv))]
        gbs = {name: round(runs[0]["kernels"][name]["bytes"] / (k[name] / 1e3) / 1e9, 1) if k[name] > 0 else None
               for name in k}
        table[f] = {"ms_total_median": round(tot[len(tot) // 2], 3), "ms_total_min": round(tot[0], 3),
                    "kernel_ms": {n: round(v, 3) for n, v in k.items()}, "kernel_GBps": gbs, "level_ms": lv,
                    "level_GBps": lgbs, "level_sparse": runs[0]["level_sparse"],
                    "level_bytes": runs[0]["level_bytes"], "level_rows": runs[0]["level_rows"]}
        print(f"flags={f:#x} total {tot[len(tot) // 2]:.2f} ms (min {tot[0]:.2f})  levels {lv} GB/s {lgbs}  kernels "
              f"{ {n: round(v, 2) for n, v in k.items()} }", flush=True)
    print(json.dumps({"level_new": ref_new, "variants": table}))


if __name__ == "__main__":
    main()
