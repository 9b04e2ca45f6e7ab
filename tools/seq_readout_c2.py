#!/usr/bin/env python3
"""Config-2 drop-in call split into the sequence call / caller-array allocation / pair readout, and the
same readout again into the now-touched arrays (page-fault cost), per call.

  python tools/seq_readout_c2.py [--reps 3]        (HGX_READOUT_THP=0: without the huge-page hint)
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
    args = ap.parse_args()
    import hypergraphdb_amd as H
    from hypergraphdb_amd import synth
    from hypergraphdb_amd._lib import check, lib, ptr
    try:
        print("thp:", open("/sys/kernel/mm/transparent_hugepage/enabled").read().strip(), flush=True)
    except OSError:
        print("thp: (unreadable)")
    g = synth.config2()
    snap = H.HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    seeds = np.asarray(g["seeds"][:64], np.int32)
    opts = H.DefaultALGenerator(snap).options()
    for i in range(args.reps + 1):
        h = C.c_void_p()
        t0 = time.perf_counter()
        check(lib().hgx_bfs_sequence(snap.handle, ptr(seeds), len(seeds), 2, C.byref(opts), C.byref(h)))
        t1 = time.perf_counter()
        ns, npairs, nl = C.c_int32(), C.c_int64(), C.c_int32()
        check(lib().hgx_seq_result_info(h, C.byref(ns), C.byref(npairs), C.byref(nl)))
        n = npairs.value
        arrs = [np.empty(n, np.int32) for _ in range(3)]
        t2 = time.perf_counter()
        check(lib().hgx_seq_result_pairs(h, *(ptr(a) for a in arrs)))
        t3 = time.perf_counter()
        check(lib().hgx_seq_result_pairs(h, *(ptr(a) for a in arrs)))
        t4 = time.perf_counter()
        lib().hgx_seq_result_free(h)
        print(f"call {i}: sequence {1e3 * (t1 - t0):.1f} ms, alloc {1e3 * (t2 - t1):.2f}, readout {1e3 * (t3 - t2):.1f}, "
              f"readout again {1e3 * (t4 - t3):.1f} ({n} pairs)", flush=True)
        del arrs
    snap.close()


if __name__ == "__main__":
    main()
