#!/usr/bin/env python3
"""Order-exact sequence (the drop-in) on config 2: 64 sources to depth 2, device time and wall time
per call (what bench.py's dropin.config2 leg runs).

  python tools/seq_c2.py [--reps 3]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--no-read", action="store_true",
                    help="free each result without reading its pairs (device time without the caller's readout)")
    args = ap.parse_args()
    import hypergraphdb_amd as H
    from hypergraphdb_amd import synth
    g = synth.config2()
    snap = H.HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    snap.set_timing(True)
    seeds = np.asarray(g["seeds"][:64], np.int32)
    ref = None
    if args.no_read:
        import ctypes as C
        from hypergraphdb_amd import _lib
        from hypergraphdb_amd._lib import check, lib, ptr
        opts = H.DefaultALGenerator(snap).options()
        for i in range(args.reps + 1):
            t0 = time.perf_counter()
            h = C.c_void_p()
            check(lib().hgx_bfs_sequence(snap.handle, ptr(seeds), len(seeds), 2, C.byref(opts), C.byref(h)))
            tr = (time.perf_counter() - t0) * 1e3
            ms, tv, bl, pl = C.c_double(), C.c_double(), C.c_double(), C.c_int64()
            check(lib().hgx_seq_result_stats(h, C.byref(ms), C.byref(tv)))   # waits for the copies
            ml = C.c_double()
            check(lib().hgx_seq_result_level_stats(h, C.byref(ml), C.byref(bl), C.byref(pl)))
            tw = (time.perf_counter() - t0) * 1e3
            lib().hgx_seq_result_free(h)
            print(f"call {i} (no readout): returned {tr:.1f} ms, copies done {tw:.1f} ms, device {ms.value:.1f} ms "
                  f"(level engine {ml.value:.1f} ms)", flush=True)
        snap.close()
        return
    for i in range(args.reps + 1):
        t0 = time.perf_counter()
        r = H.bfs_sequence(snap, seeds, 2)
        wall = (time.perf_counter() - t0) * 1e3
        n = int(r.offsets[-1])
        if ref is None:
            ref = (n, r.traversed_edges, r.atoms[:1000].copy())
        else:
            assert n == ref[0] and r.traversed_edges == ref[1] and np.array_equal(r.atoms[:1000], ref[2])
        print(f"call {i}: wall {wall:.1f} ms, device {r.ms_total:.1f} ms (level engine {r.ms_level:.1f} ms, "
              f"{r.bytes_level / 1e9:.2f} GB algorithmic, {r.pull_levels} pull levels), pairs {n}, "
              f"traversed {r.traversed_edges:.3e}", flush=True)
        del r
    snap.close()


if __name__ == "__main__":
    main()
