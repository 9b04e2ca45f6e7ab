#!/usr/bin/env python3
"""Order-exact traversal (hgx_bfs_sequence, what HGGpuTraversal.next() and the hg.subsumed /
hg.subsumes drop-ins run) on config 5: batched 1024-closure calls and single-seed latency per
direction, for the workgroup-per-seed engine (HGX_OPT_SEQ_ENGINE 0) and the level-synchronous one (1).

  python tools/seq_c5.py [--scale 1.0] [--single 200] [--engines 0,1] [--direction subsumed|subsumes]
  python tools/seq_c5.py --concurrent 40     (bench.py's drop-in step: both directions side by side on
                                              the snapshot and an execution context, median ms a step)
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--single", type=int, default=200)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--engines", default="0,1")
    ap.add_argument("--direction", choices=("both", "subsumed", "subsumes"), default="both",
                    help="one direction only (its own PMC passes: bench.py's per-direction drop-in rooflines)")
    ap.add_argument("--concurrent", type=int, default=0, help="steps of the two-context drop-in step")
    ap.add_argument("--breakdown", type=int, default=0, help="calls per direction: C call vs readout times")
    ap.add_argument("--set-first", type=int, default=0, help="--concurrent: set steps run before (bench.py's order)")
    ap.add_argument("--keep", action="store_true", help="--concurrent: keep each step's results until the next one ends")
    args = ap.parse_args()
    import hypergraphdb_amd as H
    from hypergraphdb_amd import AtomTypeCondition, DefaultALGenerator, _lib, bfs_sequence, synth
    g = synth.config5(scale=args.scale)
    snap = H.HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    snap.set_timing(True)
    T = g["subsumes_type"]
    out = {"workload": f"config5 scale {args.scale}", "seeds": len(g["seeds"]), "engines": {}}
    if args.breakdown:   # host side of a batched call per direction: the C call vs the readout into arrays
        import ctypes as C
        from hypergraphdb_amd.algorithms import SequenceResult
        from hypergraphdb_amd._lib import check, lib, ptr
        snap.set_timing(False)
        s_ = np.ascontiguousarray(g["seeds"], np.int32)
        for rev, name in ((False, "subsumed"), (True, "subsumes")):
            gen_ = DefaultALGenerator(snap, AtomTypeCondition(T), None, False, True, rev)
            opts = gen_.options()
            tc, tr = [], []
            for it in range(args.breakdown + 3):
                h = C.c_void_p()
                t0 = time.perf_counter()
                check(lib().hgx_bfs_sequence(snap.handle, ptr(s_), len(s_), _lib.HGX_UNBOUNDED, C.byref(opts), C.byref(h)))
                t1 = time.perf_counter()
                SequenceResult(h, s_)
                t2 = time.perf_counter()
                if it >= 3:
                    tc.append(t1 - t0)
                    tr.append(t2 - t1)
            out[name] = {"call_ms_median": round(float(np.median(tc)) * 1e3, 3),
                         "readout_ms_median": round(float(np.median(tr)) * 1e3, 3)}
        print(json.dumps(out))
        return
    if args.concurrent:
        from concurrent.futures import ThreadPoolExecutor
        snap.set_timing(False)
        views = [snap, snap.context()]
        gens = [DefaultALGenerator(v, AtomTypeCondition(T), None, False, True, rev) for v, rev in zip(views, (False, True))]
        pool = ThreadPoolExecutor(1)

        def step():
            f = pool.submit(bfs_sequence, views[1], g["seeds"], None, gens[1])
            a = bfs_sequence(views[0], g["seeds"], None, gens[0])
            return a, f.result()

        if args.set_first:   # bench.py's order: the set step (hgx_bfs_batch, both directions) runs first
            def set_step():
                f = pool.submit(H.bfs_batch, views[1], g["seeds"], None, gens[1])
                a = H.bfs_batch(views[0], g["seeds"], None, gens[0])
                b = f.result()
                return int(a.counts()[:, 1:].sum()) + int(b.counts()[:, 1:].sum())
            for _ in range(args.set_first):
                set_step()
        for _ in range(5):
            step()
        ts = []
        got = None
        for _ in range(args.concurrent):
            t0 = time.perf_counter()
            if args.keep:   # bench.py's loop: the previous step's result arrays stay alive during the step
                got = step()
            else:
                step()
            ts.append(time.perf_counter() - t0)
        del got
        ts.sort()
        out["concurrent_ms_per_step"] = {"median": round(ts[len(ts) // 2] * 1e3, 3), "min": round(ts[0] * 1e3, 3),
                                         "mean": round(float(np.mean(ts)) * 1e3, 3), "steps": len(ts)}
        print(json.dumps(out))
        return
    for eng in [int(x) for x in args.engines.split(",")]:
        snap.set_option(_lib.HGX_OPT_SEQ_ENGINE, eng)
        e = {}
        for rev, name in ((False, "subsumed"), (True, "subsumes")):
            if args.direction not in ("both", name):
                continue
            gen_ = DefaultALGenerator(snap, AtomTypeCondition(T), None, False, True, rev)
            bfs_sequence(snap, g["seeds"], None, gen_)   # warm-up (tables, buffers)
            walls, devs = [], []
            for _ in range(args.reps):
                t0 = time.perf_counter()
                r = bfs_sequence(snap, g["seeds"], None, gen_)
                walls.append(time.perf_counter() - t0)
                devs.append(r.ms_total)
            pairs = int(r.offsets[-1])
            singles = []
            for s in g["seeds"][: args.single]:
                t0 = time.perf_counter()
                bfs_sequence(snap, [s], None, gen_)
                singles.append(time.perf_counter() - t0)
            singles.sort()
            e[name] = {"batch_wall_ms": round(float(np.median(walls)) * 1e3, 3),
                       "batch_device_ms": round(float(np.median(devs)), 3), "pairs": pairs,
                       "traversed_items": r.traversed_edges, "ms_block": round(r.ms_block, 3),
                       "seeds_block": r.n_block, "seeds_level": r.n_level, "seeds_grid": r.n_coop,
                       "ms_grid": round(r.ms_coop, 3), "ms_level": round(r.ms_level, 3),
                       "single_ms_median": round(singles[len(singles) // 2] * 1e3, 4) if singles else None,
                       "single_ms_p90": round(singles[int(len(singles) * 0.9)] * 1e3, 4) if singles else None,
                       "single_ms_max": round(singles[-1] * 1e3, 4) if singles else None}
            print(f"engine {eng} {name}: {e[name]}", file=sys.stderr, flush=True)
        out["engines"][str(eng)] = e
    snap.set_option(_lib.HGX_OPT_SEQ_ENGINE, 0)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
