#!/usr/bin/env python3
"""Per-level row counters of the config-2 batched BFS (what each dense kernel read).

  python tools/level_rows.py [--scale 1.0] [--flags 0x3BE]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

NAMES = ["active_links", "active_pins", "inc_light", "vis_light", "new_light", "inc_heavy", "acc_hub", "new_hub"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--flags", default="0x3BE")
    args = ap.parse_args()
    import hypergraphdb_amd as H
    from hypergraphdb_amd import _lib, synth
    g = synth.config2(scale=args.scale)
    deg = np.bincount(g["tgt_idx"], minlength=g["num_atoms"])
    heavy = deg > 512
    print(json.dumps({"I": int(deg.sum()), "I_heavy": int(deg[heavy].sum()), "n_heavy": int(heavy.sum())}), flush=True)
    snap = H.HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    snap.set_timing(True)
    snap.set_option(_lib.HGX_OPT_BFS_FLAGS, int(args.flags, 0))
    for _ in range(2):
        r = H.bfs_batch(snap, g["seeds"], g["depth"])
        st = r.stats(accounting=True)
        r.close()
    for d, rows in enumerate(st["level_rows"]):
        print(json.dumps({"level": d, "ms": st["level_ms"][d], "new": st["level_new"][d],
                          **{k: v for k, v in zip(NAMES, rows)}}), flush=True)
    print(json.dumps({k: round(v["ms"], 3) for k, v in st["kernels"].items()}), flush=True)


if __name__ == "__main__":
    main()
