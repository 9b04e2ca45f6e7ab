#!/usr/bin/env python3
"""Per-query candidate counts of the config-3 bench batch (the type-T slice of the anchor with the
fewest incident links -- what one query of the fused pattern kernel scans), and the fused kernel's
time against the batch size.

  python tools/pattern_slices.py [--scale 1.0]
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
    ap.add_argument("--scale", type=float, default=1.0)
    args = ap.parse_args()
    import hypergraphdb_amd as H
    from hypergraphdb_amd import synth
    from hypergraphdb_amd.query import pattern_batch_arrays
    g = synth.config3(scale=args.scale)
    Q = g["queries"]
    t0 = time.time()
    deg = np.bincount(g["tgt_idx"], minlength=g["num_atoms"])
    order = np.argsort(g["tgt_idx"], kind="stable")
    off = np.concatenate([[0], np.cumsum(deg)])
    link_of_pin = np.repeat(np.arange(len(g["link_type"]), dtype=np.int64), np.diff(g["tgt_off"]))
    n = len(Q["type"])
    nc = np.zeros(n, np.int64)
    mind = np.zeros(n, np.int64)
    for q in range(n):
        anchors = {int(Q["a"][q]), int(Q["x"][q]), int(Q["y"][q])}
        best = min(anchors, key=lambda a: (deg[a], a))
        mind[q] = deg[best]
        links = link_of_pin[order[off[best]:off[best + 1]]]
        nc[q] = int((g["link_type"][links] == Q["type"][q]).sum())
    print(json.dumps({"host_s": round(time.time() - t0, 1), "candidates_total": int(nc.sum()),
                      "max": int(nc.max()), "p99": float(np.percentile(nc, 99)), "p50": float(np.median(nc)),
                      "over_1024": int((nc > 1024).sum()), "min_anchor_degree_max": int(mind.max()),
                      "min_anchor_degree_p99": float(np.percentile(mind, 99))}), flush=True)
    snap = H.HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    snap.set_timing(True)
    for m in (1000, 5000, 10000):
        sel = np.arange(m)
        packed = (Q["type"][sel], np.arange(m + 1, dtype=np.int64), Q["a"][sel], np.ones(m, np.int32),
                  np.arange(0, 3 * m + 1, 3, dtype=np.int64),
                  np.stack([Q["x"][sel], np.full(m, -1, np.int32), Q["y"][sel]], 1).reshape(-1))
        ms = []
        for _ in range(5):
            r = pattern_batch_arrays(snap, *packed)
            ms.append(r.ms["ms_match"])
        big = np.argsort(-nc[:m])[:3]
        print(json.dumps({"queries": m, "match_ms": sorted(ms)[2], "largest_slices": nc[big].tolist()}), flush=True)
    # the largest-slice queries alone
    for k in (1, 10):
        sel = np.argsort(-nc)[:k]
        m = len(sel)
        packed = (Q["type"][sel], np.arange(m + 1, dtype=np.int64), Q["a"][sel], np.ones(m, np.int32),
                  np.arange(0, 3 * m + 1, 3, dtype=np.int64),
                  np.stack([Q["x"][sel], np.full(m, -1, np.int32), Q["y"][sel]], 1).reshape(-1))
        ms = []
        for _ in range(5):
            r = pattern_batch_arrays(snap, *packed)
            ms.append(r.ms["ms_match"])
        print(json.dumps({"largest_k": k, "match_ms": sorted(ms)[2], "slices": nc[sel].tolist()}), flush=True)


if __name__ == "__main__":
    main()
