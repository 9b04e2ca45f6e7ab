#!/usr/bin/env python3
"""Quality of the vertex-cut link placement (hgx_partition_plan) on config 4 at a given scale:
remote holders per present atom (the rows one dense level exchanges, per direction, divided by the
present atoms) and the pin balance, for the greedy plan and for a random placement.

  python tools/vcut_quality.py --scale 0.1 --parts 8
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def remote_per_present(g, plan, NP):
    ar = np.diff(g["tgt_off"])
    pairs = np.unique(g["tgt_idx"].astype(np.int64) * NP + np.repeat(plan, ar).astype(np.int64))
    present = len(np.unique(g["tgt_idx"]))
    return (len(pairs) - present) / present, present


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=0.1)
    ap.add_argument("--parts", type=int, default=8)
    args = ap.parse_args()
    from hypergraphdb_amd import synth
    from hypergraphdb_amd.partition import partition_plan
    g = synth.config4(scale=args.scale, n_sources=64)
    t0 = time.time()
    plan = partition_plan(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"], args.parts)
    t_plan = time.time() - t0
    ar = np.diff(g["tgt_off"])
    load = np.bincount(plan, weights=ar, minlength=args.parts)
    rg, present = remote_per_present(g, plan, args.parts)
    rnd = np.random.default_rng(1).integers(0, args.parts, len(plan)).astype(np.int32)
    rr, _ = remote_per_present(g, rnd, args.parts)
    print(json.dumps({"scale": args.scale, "parts": args.parts, "links": len(plan), "pins": int(ar.sum()),
                      "present_atoms": present, "plan_seconds": round(t_plan, 2),
                      "remote_per_present_greedy": round(rg, 4), "remote_per_present_random": round(rr, 4),
                      "pin_load_max_over_mean": round(float(load.max() / load.mean()), 4)}))


if __name__ == "__main__":
    main()
