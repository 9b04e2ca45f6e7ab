#!/usr/bin/env python3
"""Source tiling A/B for the config-2 headline step (VERDICT r5 'do this' 2).

  python tools/ab_tiles.py --tiles 1,2,4,8,16 --rounds 3

The 1024-source batch runs as k tiles of 1024/k sources, one hgx_bfs_batch per tile (S/k sources ->
rows of S/k/8 bytes, so the per-atom source-mask table shrinks to 10M x 128/k B: 160 MB at k = 8,
inside the 256 MiB Infinity Cache).  Every tile re-reads the CSR.  Prints the summed device ms of the
k tiles (median over rounds, interleaved), the per-kernel split, and checks that the concatenated
per-source per-depth counts and the summed TEPS numerator equal the one-batch run's.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", default="1,2,4,8,16")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--sources", type=int, default=1024)
    ap.add_argument("--depth", type=int, default=4)
    args = ap.parse_args()
    import numpy as np
    import hypergraphdb_amd as H
    from hypergraphdb_amd import synth
    g = synth.config2(scale=args.scale, n_sources=args.sources)
    snap = H.HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    snap.set_timing(True)
    seeds = np.asarray(g["seeds"], np.int32)
    ks = [int(k) for k in args.tiles.split(",")]
    res = {k: [] for k in ks}
    ref_counts = ref_tr = None
    for r in range(args.rounds + 1):
        for k in ks:
            n = len(seeds) // k
            ms, tr, kern, counts = 0.0, 0.0, {}, []
            for t in range(k):
                out = H.bfs_batch(snap, seeds[t * n:(t + 1) * n], args.depth)
                st = out.stats(accounting=(r == 0))
                ms += st["ms_total"]
                if r == 0:
                    tr += st["traversed_edges"]
                    counts.append(out.counts())
                for name, v in st["kernels"].items():
                    kern[name] = kern.get(name, 0.0) + v["ms"]
                out.close()
            if r == 0:
                w = max(c.shape[1] for c in counts)
                cc = np.concatenate([np.pad(c, ((0, 0), (0, w - c.shape[1]))) for c in counts])
                if ref_counts is None:
                    ref_counts, ref_tr = cc, tr
                assert cc.shape == ref_counts.shape and (cc == ref_counts).all(), (k, "per-source counts")
                assert tr == ref_tr, (k, tr, ref_tr)
            else:
                res[k].append((ms, kern))
    out = {}
    for k in ks:
        runs = sorted(res[k], key=lambda x: x[0])
        ms, kern = runs[len(runs) // 2]
        out[k] = {"device_ms": round(ms, 3), "teps": ref_tr / (ms / 1e3),
                  "kernel_ms": {n: round(v, 3) for n, v in kern.items() if v > 0}}
        print(f"tiles={k:2d} ({len(seeds) // k} sources each): device {ms:.2f} ms  {ref_tr / (ms / 1e3):.3e} TEPS  "
              f"{out[k]['kernel_ms']}", flush=True)
    print(json.dumps({"traversed_edges": ref_tr, "tiles": out}))


if __name__ == "__main__":
    main()
