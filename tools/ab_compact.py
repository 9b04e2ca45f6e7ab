#!/usr/bin/env python3
"""A/B: config 2 on the whole snapshot (atom space = all 50M atoms) vs a one-part shard (atom space
compacted to the atoms with incidence).  Same seeds, identical counts required.

  python tools/ab_compact.py --rounds 3
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--config", type=int, default=2)
    args = ap.parse_args()
    import hypergraphdb_amd as H
    from hypergraphdb_amd import synth
    from hypergraphdb_amd.partition import Shard, ShardSnapshot, pbfs_batch_group
    g = synth.config2(scale=args.scale) if args.config == 2 else synth.config4(scale=args.scale)
    whole = H.HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    sh = Shard.build(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"], 1, 0)
    part = ShardSnapshot(sh, 0)
    print(f"A={g['num_atoms']} local={sh.n_local}", flush=True)
    sh.close()
    whole.set_timing(True)
    part.set_timing(True)
    c0 = H.bfs_batch(whole, g["seeds"], 4).counts()
    c1 = pbfs_batch_group([part], g["seeds"], 4).counts()
    assert np.array_equal(c0, c1)
    for r in range(args.rounds):
        for name, run in (("whole", lambda: H.bfs_batch(whole, g["seeds"], 4)),
                          ("compact", lambda: pbfs_batch_group([part], g["seeds"], 4).parts[0])):
            res = run()
            st = res.stats(accounting=False)
            res.close()
            print(name, round(st["ms_total"], 3), st["level_ms"],
                  {k: round(v["ms"], 2) for k, v in st["kernels"].items()}, flush=True)


if __name__ == "__main__":
    main()
