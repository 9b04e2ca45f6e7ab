#!/usr/bin/env python3
"""Host time of an order-exact result's readout on config 5 (the drop-in's batched 1024 closures, one
direction): the hgx_bfs_sequence call, then each hgx_seq_result_* call the Python mirror makes.

  python tools/seq_readout_c5.py [--reps 3] [--reverse]
"""
import argparse
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--reverse", action="store_true", help="hg.subsumes (default hg.subsumed)")
    args = ap.parse_args()
    import hypergraphdb_amd as H
    from hypergraphdb_amd import AtomTypeCondition, DefaultALGenerator, synth
    from hypergraphdb_amd._lib import check, lib, ptr
    g = synth.config5()
    snap = H.HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    st = int(g["subsumes_type"])
    gen = DefaultALGenerator(snap, AtomTypeCondition(st), None, False, True, args.reverse)   # as bench.py
    opts = gen.options()
    seeds = np.asarray(g["seeds"], np.int32)
    L = lib()
    for rep in range(args.reps + 1):
        t = [time.perf_counter()]
        h = C.c_void_p()
        check(L.hgx_bfs_sequence(snap.handle, ptr(seeds), len(seeds), -1, C.byref(opts), C.byref(h)))
        t.append(time.perf_counter())
        ns, npairs, nl = C.c_int32(), C.c_int64(), C.c_int32()
        check(L.hgx_seq_result_info(h, C.byref(ns), C.byref(npairs), C.byref(nl)))
        off = np.zeros(len(seeds) + 1, np.int64)
        check(L.hgx_seq_result_offsets(h, ptr(off)))
        t.append(time.perf_counter())
        n = npairs.value
        a = [np.empty(max(n, 1), np.int32) for _ in range(3)]
        t.append(time.perf_counter())
        check(L.hgx_seq_result_pairs(h, ptr(a[0]), ptr(a[1]), ptr(a[2])))
        t.append(time.perf_counter())
        L.hgx_seq_result_free(h)
        t.append(time.perf_counter())
        d = [1e3 * (t[i + 1] - t[i]) for i in range(len(t) - 1)]
        print(f"rep {rep}: call {d[0]:.3f} ms, info+offsets {d[1]:.3f}, alloc {d[2]:.3f}, pairs {d[3]:.3f}, "
              f"free {d[4]:.3f} ({n} pairs)", flush=True)
    snap.close()


if __name__ == "__main__":
    main()
