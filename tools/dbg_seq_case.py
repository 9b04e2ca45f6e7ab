#!/usr/bin/env python3
"""Debug: one order-exact case (tests/test_gpu_seq.py::test_power_law_hubs_and_chunking's first call) against
the oracle, with the engine split (workgroup / grid stage / level engine, pull levels).

  [HGX_LIB_VARIANT=<name>] python tools/dbg_seq_case.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import hypergraphdb_amd as H
    from hypergraphdb_amd import _lib, synth
    from oracle_ctypes import OracleGraph, algen
    g = synth.hypergraph(3000, 20000, 2, 8, 2.1, 3, seed=21)
    snap = H.HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    orc = OracleGraph(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    seeds = np.concatenate([np.arange(4), np.arange(2950, 3000)]).astype(np.int32)
    for eng in (0, 2):
        for pull in (0, 1, 2):
            snap.set_option(_lib.HGX_OPT_SEQ_ENGINE, eng)
            snap.set_option(_lib.HGX_OPT_SEQ_PULL, pull)
            r = H.bfs_sequence(snap, seeds, 3)
            bad = []
            for i, s in enumerate(seeds):
                l_, a, d, _ = orc.bfs(int(s), 3, algen(-1, True, True, False, False))
                gl, ga, gd = r.pairs(i)
                if not (np.array_equal(ga, a) and np.array_equal(gl, l_) and np.array_equal(gd, d)):
                    bad.append((i, len(ga), len(a)))
            print(f"engine {eng} pull {pull}: block {r.n_block} grid {r.n_coop} level {r.n_level} pull_levels "
                  f"{r.pull_levels}: {'ok' if not bad else 'BAD ' + str(bad[:6])}", flush=True)


if __name__ == "__main__":
    main()
