#!/usr/bin/env python3
"""Host-side split of one config-5 direction (hg.subsumed closures of 1024 classes): wall time of the
traversal call, the readout, the stats call and the release, medians over the calls.

  python tools/c5_host.py [--scale 1.0] [--calls 30] [--timing]
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
    ap.add_argument("--timing", action="store_true", help="device events per level (as the bench)")
    args = ap.parse_args()
    import hypergraphdb_amd as H
    from hypergraphdb_amd import AtomTypeCondition, DefaultALGenerator, synth
    g = synth.config5(scale=args.scale, n_sources=1024)
    snap = H.HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    snap.set_timing(args.timing)
    for rev in (False, True):
        gen = DefaultALGenerator(snap, AtomTypeCondition(g["subsumes_type"]), None, False, True, rev)
        ph = {k: [] for k in ("bfs_batch", "counts", "stats", "close", "total")}
        for i in range(args.calls + 3):
            t0 = time.perf_counter()
            r = H.bfs_batch(snap, g["seeds"], None, gen)
            t1 = time.perf_counter()
            r.counts()
            t2 = time.perf_counter()
            st = r.stats(accounting=False, raw=True)
            t3 = time.perf_counter()
            r.close()
            t4 = time.perf_counter()
            if i >= 3:
                for k, a, b in (("bfs_batch", t0, t1), ("counts", t1, t2), ("stats", t2, t3), ("close", t3, t4),
                                ("total", t0, t4)):
                    ph[k].append((b - a) * 1e3)
        d = st.as_dict()
        print(f"[c5 host] reverse={rev} levels {d.get('n_levels_expanded')} device ms {d.get('ms_total', 0):.3f}; " +
              ", ".join(f"{k} {np.median(v):.3f}" for k, v in ph.items()) + " ms (medians)")


if __name__ == "__main__":
    main()
