#!/usr/bin/env python3
"""Per-level breakdown of the config-5 subsumption closures (both directions).

  python tools/ab_c5.py [--scale 1.0] [--flags 0x3BE]
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
    ap.add_argument("--flags", default="0x3BE")
    ap.add_argument("--sources", type=int, default=1024)
    ap.add_argument("--push", default="0", help="HGX_OPT_PUSH_BATCH values (only 0 remains: one wavefront per atom)")
    args = ap.parse_args()
    import hypergraphdb_amd as H
    from hypergraphdb_amd import AtomTypeCondition, DefaultALGenerator, _lib, synth
    g = synth.config5(scale=args.scale, n_sources=args.sources)
    snap = H.HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    snap.set_timing(True)
    for f, pb in [(f, pb) for f in args.flags.split(",") for pb in args.push.split(",")]:
        snap.set_option(_lib.HGX_OPT_BFS_FLAGS, int(f, 0))
        snap.set_option(_lib.HGX_OPT_PUSH_BATCH, int(pb))
        for rev in (False, True):
            gen = DefaultALGenerator(snap, AtomTypeCondition(g["subsumes_type"]), None, False, True, rev)
            for _ in range(2):
                r = H.bfs_batch(snap, g["seeds"], None, gen)
                st = r.stats(accounting=True)
                r.close()
            t0 = time.perf_counter()
            for _ in range(5):
                H.bfs_batch(snap, g["seeds"], None, gen).close()
            wall = (time.perf_counter() - t0) / 5 * 1e3
            print(json.dumps({"flags": f, "push_batch": int(pb), "reverse": rev, "ms_total": round(st["ms_total"], 3),
                              "wall_ms": round(wall, 3),
                              "kernels": {k: round(v["ms"], 3) for k, v in st["kernels"].items()},
                              "level_ms": st["level_ms"], "level_new": st["level_new"],
                              "level_sparse": st["level_sparse"], "union_frontier": st["union_frontier"]}), flush=True)


if __name__ == "__main__":
    main()
