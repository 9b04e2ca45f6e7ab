#!/usr/bin/env python3
"""Per-call wall time vs device time of one config-3 pattern batch (host-overhead check).

  python tools/pattern_timing.py [--scale 1.0] [--calls 30]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--calls", type=int, default=30)
    ap.add_argument("--queries", type=int, default=10_000)
    args = ap.parse_args()
    import hypergraphdb_amd as H
    from hypergraphdb_amd import synth
    from hypergraphdb_amd.query import pattern_batch_arrays
    g = synth.config3(scale=args.scale, n_queries=args.queries)
    Q = g["queries"]
    snap = H.HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    snap.set_timing(True)
    nq = len(Q["type"])
    packed = (Q["type"], np.arange(nq + 1, dtype=np.int64), Q["a"], np.ones(nq, np.int32),
              np.arange(0, 3 * nq + 1, 3, dtype=np.int64),
              np.stack([Q["x"], np.full(nq, -1, np.int32), Q["y"]], 1).reshape(-1))
    walls, devs = [], []
    for i in range(args.calls):
        t0 = time.perf_counter()
        r = pattern_batch_arrays(snap, *packed)
        walls.append((time.perf_counter() - t0) * 1e3)
        devs.append(r.ms["ms_total"])
    w, d = np.array(walls[3:]), np.array(devs[3:])
    print(f"wall ms: median {np.median(w):.3f} min {w.min():.3f} max {w.max():.3f}; "
          f"device ms: median {np.median(d):.3f}; match ms {r.ms['ms_match']:.3f}; results {int(r.offsets[-1])}")
    print("walls", [round(x, 3) for x in walls])


if __name__ == "__main__":
    main()
