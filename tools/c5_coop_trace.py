#!/usr/bin/env python3
"""Per-level trace of the multi-workgroup stage on config 5's big hg.subsumed closures (HGX_CO_TRACE).

  HGX_CO_TRACE=1 python tools/c5_coop_trace.py
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import hypergraphdb_amd as H
    from hypergraphdb_amd import AtomTypeCondition, DefaultALGenerator, _lib, synth
    g = synth.config5()
    snap = H.HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    gen = DefaultALGenerator(snap, AtomTypeCondition(g["subsumes_type"]), None, False, True, False)
    r = H.bfs_batch(snap, g["seeds"], None, gen)
    size = r.counts()[:, 1:].sum(1)
    r.close()
    big = np.ascontiguousarray(g["seeds"][size > 1534])
    print("big closures", sorted(size[size > 1534].tolist()), flush=True)
    snap.set_option(_lib.HGX_OPT_BFS_BLOCK, 2)   # straight to the multi-workgroup stage
    for _ in range(3):
        t0 = time.perf_counter()
        r = H.bfs_batch(snap, big, None, gen)
        r.counts()
        st = r.stats(accounting=False)
        r.close()
        print(f"wall {(time.perf_counter() - t0) * 1e3:.3f} ms, coop seeds {st['block_coop']}", flush=True)
    snap.close()


if __name__ == "__main__":
    main()
