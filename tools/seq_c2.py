#!/usr/bin/env python3
"""Order-exact sequence (the drop-in) on config 2: 64 sources to depth 2, device time and wall time
per call (what bench.py's dropin.config2 leg runs).

  python tools/seq_c2.py [--reps 3]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import hypergraphdb_amd as H
    from hypergraphdb_amd import synth
    g = synth.config2()
    snap = H.HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    snap.set_timing(True)
    seeds = np.asarray(g["seeds"][:64], np.int32)
    ref = None
    for i in range(args.reps + 1):
        t0 = time.perf_counter()
        r = H.bfs_sequence(snap, seeds, 2)
        wall = (time.perf_counter() - t0) * 1e3
        n = int(r.offsets[-1])
        if ref is None:
            ref = (n, r.traversed_edges, r.atoms[:1000].copy())
        else:
            assert n == ref[0] and r.traversed_edges == ref[1] and np.array_equal(r.atoms[:1000], ref[2])
        print(f"call {i}: wall {wall:.1f} ms, device {r.ms_total:.1f} ms (level engine {r.ms_level:.1f} ms, "
              f"{r.bytes_level / 1e9:.2f} GB algorithmic, {r.pull_levels} pull levels), pairs {n}, "
              f"traversed {r.traversed_edges:.3e}", flush=True)
        del r
    snap.close()


if __name__ == "__main__":
    main()
