#!/usr/bin/env python3
"""Per-call wall time vs device time of one config-3 pattern batch (host-overhead check).

  python tools/pattern_timing.py [--scale 1.0] [--calls 30]
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
    ap.add_argument("--queries", type=int, default=10_000)
    ap.add_argument("--fused", default="0", help="HGX_OPT_QUERY_FUSED values to compare, interleaved (e.g. 1,0)")
    ap.add_argument("--inline", default="1", help="HGX_OPT_QUERY_INLINE values to compare, interleaved (e.g. 1,0)")
    ap.add_argument("--flat", default="2", help="HGX_OPT_QUERY_FLAT values to compare, interleaved (e.g. 2,1,0)")
    ap.add_argument("--no-timing", action="store_true", help="no device events (wall time without their gaps)")
    ap.add_argument("--resident", action="store_true",
                    help="run the batch as a resident query set (hgx_query_set_create + hgx_pattern_batch_set)")
    args = ap.parse_args()
    import hypergraphdb_amd as H
    from hypergraphdb_amd import synth
    from hypergraphdb_amd.query import QuerySet, pattern_batch_arrays
    g = synth.config3(scale=args.scale, n_queries=args.queries)
    Q = g["queries"]
    snap = H.HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    snap.set_timing(not args.no_timing)
    nq = len(Q["type"])
    packed = (Q["type"], np.arange(nq + 1, dtype=np.int64), Q["a"], np.ones(nq, np.int32),
              np.arange(0, 3 * nq + 1, 3, dtype=np.int64),
              np.stack([Q["x"], np.full(nq, -1, np.int32), Q["y"]], 1).reshape(-1))
    from hypergraphdb_amd import _lib
    opts = [(int(f), int(i), int(fl)) for f in args.fused.split(",") for i in args.inline.split(",")
            for fl in args.flat.split(",")]
    walls = {o: [] for o in opts}
    devs = {o: [] for o in opts}
    match = {o: [] for o in opts}
    gbs = {o: [] for o in opts}
    ref = None
    qset = None
    for i in range(args.calls):
        for o in opts:
            snap.set_option(_lib.HGX_OPT_QUERY_FUSED, o[0])
            snap.set_option(_lib.HGX_OPT_QUERY_INLINE, o[1])
            snap.set_option(_lib.HGX_OPT_QUERY_FLAT, o[2])
            if args.resident and qset is None:
                qset = QuerySet(snap, *packed)
            t0 = time.perf_counter()
            r = qset.run(snap) if args.resident else pattern_batch_arrays(snap, *packed)
            walls[o].append((time.perf_counter() - t0) * 1e3)
            devs[o].append(r.ms["ms_total"])
            match[o].append(r.ms["ms_match"])
            gbs[o].append(r.ms["bytes_match"] / max(r.ms["ms_match"], 1e-9) / 1e6)
            if ref is None:
                ref = (r.offsets.copy(), r.ids.copy())
            elif i < 2:
                assert np.array_equal(ref[0], r.offsets) and np.array_equal(ref[1], r.ids), "paths differ"
    if args.resident:
        # the same set into caller buffers (hgx_pattern_batch_set_into): no result object per batch
        off = np.zeros(len(ref[0]), np.int64)
        ids = np.zeros(len(ref[1]) + 1, np.int32)
        wi = []
        for i in range(args.calls):
            t0 = time.perf_counter()
            n = qset.run_into(snap, off, ids)
            wi.append((time.perf_counter() - t0) * 1e3)
            assert n == len(ref[1]) and np.array_equal(off, ref[0]) and np.array_equal(ids[:n], ref[1])
        w = np.array(wi[3:])
        print(f"into caller buffers (flat={opts[-1][2]}) wall ms: median {np.median(w):.3f} min {w.min():.3f} "
              f"max {w.max():.3f}")
    for o in opts:
        w, d, m = np.array(walls[o][3:]), np.array(devs[o][3:]), np.array(match[o][3:])
        print(f"fused,inline,flat={o} wall ms: median {np.median(w):.3f} min {w.min():.3f} max {w.max():.3f}; "
              f"device ms: median {np.median(d):.3f}; match ms median {np.median(m):.3f} "
              f"({np.median(gbs[o][3:]):.1f} GB/s algorithmic); results {int(r.offsets[-1])}")
        print("walls", [round(x, 3) for x in walls[o]])


if __name__ == "__main__":
    main()
