#!/usr/bin/env python3
"""Where the host time of a large order-exact result goes (config 2's drop-in call: 258M pairs):
the hgx_bfs_sequence call itself, then hgx_seq_result_pairs into (a) fresh numpy arrays, (b) arrays
touched beforehand, (c) fresh anonymous mappings advised MADV_HUGEPAGE.  --bfs-first runs the bench's
1024-source hgx_bfs_batch first (the bench's process state when its drop-in leg runs).

  python tools/readout_ab.py [--bfs-first] [--reps 2]
"""
import argparse
import ctypes as C
import mmap
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def huge_array(n):
    m = mmap.mmap(-1, 4 * n, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    if hasattr(mmap, "MADV_HUGEPAGE"):
        m.madvise(mmap.MADV_HUGEPAGE)
    return np.frombuffer(m, np.int32, n), m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bfs-first", action="store_true")
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    import hypergraphdb_amd as H
    from hypergraphdb_amd import _lib, synth
    from hypergraphdb_amd._lib import check, lib, ptr
    try:
        print("THP:", open("/sys/kernel/mm/transparent_hugepage/enabled").read().strip(), flush=True)
    except OSError:
        pass
    g = synth.config2()
    snap = H.HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    snap.set_timing(True)
    if args.bfs_first:
        r = H.bfs_batch(snap, g["seeds"], 4)
        r.counts()
        r.close()
    seeds = np.asarray(g["seeds"][:64], np.int32)
    opts = H.DefaultALGenerator(snap).options()
    for rep in range(args.reps + 1):
        for mode in ("fresh", "touched", "hugepage"):
            h = C.c_void_p()
            t0 = time.perf_counter()
            check(lib().hgx_bfs_sequence(snap.handle, ptr(seeds), len(seeds), 2, C.byref(opts), C.byref(h)))
            t1 = time.perf_counter()
            ns, npairs, nl = C.c_int32(), C.c_int64(), C.c_int32()
            check(lib().hgx_seq_result_info(h, C.byref(ns), C.byref(npairs), C.byref(nl)))
            n = npairs.value
            keep = []
            t2 = time.perf_counter()
            if mode == "fresh":
                arrs = [np.empty(n, np.int32) for _ in range(3)]
            elif mode == "touched":
                arrs = [np.ones(n, np.int32) for _ in range(3)]
            else:
                arrs = []
                for _ in range(3):
                    a, m = huge_array(n)
                    arrs.append(a)
                    keep.append(m)
            t3 = time.perf_counter()
            check(lib().hgx_seq_result_pairs(h, ptr(arrs[0]), ptr(arrs[1]), ptr(arrs[2])))
            t4 = time.perf_counter()
            lib().hgx_seq_result_free(h)
            print(f"rep {rep} {mode:8s}: call {1e3 * (t1 - t0):.1f} ms, alloc {1e3 * (t3 - t2):.1f} ms, pairs copy "
                  f"{1e3 * (t4 - t3):.1f} ms ({n} pairs)", flush=True)
            del arrs, keep
    snap.close()


if __name__ == "__main__":
    main()
