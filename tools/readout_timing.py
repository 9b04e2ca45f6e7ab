#!/usr/bin/env python3
"""Host wall of one batched traversal split into bfs_batch / result readout (counts) / stats + close,
for the config-5 closures (both directions) and optionally config 2.

  python tools/readout_timing.py [--c5-scale 1.0] [--config2] [--steps 5]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def split(snap, seeds, depth, gen, steps):
    import hypergraphdb_amd as H
    t = {"bfs_batch": 0.0, "counts": 0.0, "stats+close": 0.0}
    for _ in range(steps + 1):
        a = time.perf_counter()
        r = H.bfs_batch(snap, seeds, depth, gen)
        b = time.perf_counter()
        r.counts()
        c = time.perf_counter()
        r.stats(accounting=False)
        r.close()
        e = time.perf_counter()
        if _ == 0:
            continue   # warm-up
        t["bfs_batch"] += b - a
        t["counts"] += c - b
        t["stats+close"] += e - c
    return {k: round(v / steps * 1e3, 3) for k, v in t.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--c5-scale", type=float, default=1.0)
    ap.add_argument("--config2", action="store_true")
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    import hypergraphdb_amd as H
    from hypergraphdb_amd import AtomTypeCondition, DefaultALGenerator, synth
    g = synth.config5(scale=args.c5_scale)
    snap = H.HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    snap.set_timing(True)
    for rev in (False, True):
        gen = DefaultALGenerator(snap, AtomTypeCondition(g["subsumes_type"]), None, False, True, rev)
        print("config5", "subsumes" if rev else "subsumed", split(snap, g["seeds"], None, gen, args.steps), flush=True)
    snap.close()
    if args.config2:
        g = synth.config2()
        snap = H.HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
        snap.set_timing(True)
        print("config2", split(snap, g["seeds"], 4, None, args.steps), flush=True)
        snap.close()


if __name__ == "__main__":
    main()
