#!/usr/bin/env python3
"""The config-5 bench step alone (hg.subsumed + hg.subsumes closures of 1024 classes, each ending with
its readout), the two directions one after the other and side by side on two execution contexts
(hgx_graph_context), for A/B runs and kernel traces:

  python tools/c5_step.py [--scale 1.0] [--steps 20] [--mode both|serial|concurrent]
  rocprofv3 --kernel-trace --stats -d gpurun_out/prof -- python3 tools/c5_step.py --mode concurrent
"""
import argparse
import json

import numpy as np
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--mode", default="both", choices=("both", "serial", "concurrent"))
    ap.add_argument("--timing", action="store_true", help="device events per level (adds event records)")
    ap.add_argument("--split", type=int, default=1,
                    help="concurrent mode: each direction's sources in this many batches, each on its own context")
    args = ap.parse_args()
    import hypergraphdb_amd as H
    from hypergraphdb_amd import AtomTypeCondition, DefaultALGenerator, synth
    g = synth.config5(scale=args.scale, n_sources=1024)
    snap = H.HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    snap.set_timing(args.timing)
    K = max(1, args.split)
    views = [snap] + [snap.context() for _ in range(2 * K - 1)]
    T = g["subsumes_type"]
    # job j: direction j % 2 (subsumed / subsumes), source batch j // 2 of K
    gens = [DefaultALGenerator(v, AtomTypeCondition(T), None, False, True, bool(j % 2)) for j, v in enumerate(views)]
    parts = np.array_split(np.asarray(g["seeds"], np.int32), K)
    pool = ThreadPoolExecutor(2 * K - 1)

    def job(j, seeds=None):
        r = H.bfs_batch(views[j], parts[j // 2] if seeds is None else seeds, None, gens[j])
        n = int(r.counts()[:, 1:].sum())
        st = r.stats(accounting=False, raw=True)
        r.close()
        return n, st

    def step(concurrent):
        if not concurrent:
            return [job(0, g["seeds"]), job(1, g["seeds"])]
        fs = [pool.submit(job, j) for j in range(1, 2 * K)]
        res = [job(0)] + [f.result() for f in fs]
        # per direction: closure atoms summed over the source batches, the batches' stats
        return [(sum(res[j][0] for j in range(d, 2 * K, 2)), res[d][1]) for d in (0, 1)]

    out = {"tool": "tools/c5_step.py", "scale": args.scale, "steps": args.steps, "split": K}
    modes = {"both": (False, True), "serial": (False,), "concurrent": (True,)}[args.mode]
    ref = None
    for conc in modes:
        for _ in range(args.warmup):
            step(conc)
        t0 = time.perf_counter()
        res = [step(conc) for _ in range(args.steps)]
        ms = (time.perf_counter() - t0) / args.steps * 1e3
        closures = [n for n, _ in res[0]]
        if ref is None:
            ref = closures
        assert closures == ref, "closure sizes differ between modes"
        key = "concurrent" if conc else "serial"
        out[key] = {"ms_per_step": round(ms, 4), "closure_atoms": closures,
                    "levels": [st.n_levels_expanded for _, st in res[0]]}
        if args.timing:
            out[key]["device_ms"] = [round(st.ms_total, 4) for _, st in res[-1]]
        print(f"[c5] {key}: {ms:.3f} ms/step", file=sys.stderr, flush=True)
    pool.shutdown()
    for v in views[1:]:
        v.close()
    snap.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
