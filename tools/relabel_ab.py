#!/usr/bin/env python3
"""Config-2 step time under locality-ordered link numberings (VERDICT r2 'do this' 6).

Links are atoms too; renumbering them (their ranks) changes no per-depth node set, only where the
engine's link rows (tgt rows, lf rows) and incidence entries sit in HBM.  Orders:
  none  the generator's order (independent links: no locality)
  hub   links sorted by their highest-degree target (Chung-Lu node ids are in descending weight
        order, so the smallest target id): the links of one hub are contiguous
  hub2  by (smallest, second smallest) target id
Every order must give the same per-source per-depth counts; the tool reports the device ms per
level and per kernel (HIP events) of each.

  python tools/relabel_ab.py [--orders none,hub,hub2] [--steps 5] [--scale 1.0]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def relabel(g, order):
    if order == "none":
        return g
    off, tg = g["tgt_off"], g["tgt_idx"]
    ar = np.diff(off)
    M = len(ar)
    first = np.minimum.reduceat(tg, off[:-1])   # every link has >= 2 targets
    if order == "hub":
        perm = np.argsort(first, kind="stable")
    elif order == "hub2":
        # second smallest target: min over the row with the smallest masked out
        big = np.where(tg == np.repeat(first, ar), np.int32(2**31 - 1), tg)
        second = np.minimum.reduceat(big, off[:-1])
        perm = np.lexsort((second, first))
    else:
        raise ValueError(order)
    ar2 = ar[perm]
    off2 = np.zeros(M + 1, np.int64)
    np.cumsum(ar2, out=off2[1:])
    src = np.repeat(off[:-1][perm] - off2[:-1], ar2) + np.arange(off2[-1], dtype=np.int64)
    out = dict(g)
    out["tgt_off"] = off2
    out["tgt_idx"] = tg[src]
    out["link_type"] = g["link_type"][perm]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--orders", default="none,hub,hub2")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--scale", type=float, default=1.0)
    args = ap.parse_args()
    import hypergraphdb_amd as H
    from hypergraphdb_amd import synth
    base = synth.config2(scale=args.scale)
    ref = None
    out = {"tool": "tools/relabel_ab.py", "scale": args.scale, "steps": args.steps, "orders": {}}
    for order in args.orders.split(","):
        t0 = time.time()
        g = relabel(base, order)
        snap = H.HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"],
                                    keep_host=False)
        snap.set_timing(True)
        print(f"[relabel] {order}: graph + snapshot in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
        for _ in range(2):
            r = H.bfs_batch(snap, g["seeds"], 4)
            c = r.counts()
            r.close()
        if ref is None:
            ref = c.copy()
        assert np.array_equal(c, ref), f"order {order}: per-depth counts differ"
        sts = []
        t1 = time.perf_counter()
        for _ in range(args.steps):
            r = H.bfs_batch(snap, g["seeds"], 4)
            r.counts()
            sts.append(r.stats(accounting=False))
            r.close()
        wall = (time.perf_counter() - t1) / args.steps * 1e3
        n = len(sts)
        levels = [round(sum(s["level_ms"][d] for s in sts) / n, 3) for d in range(len(sts[0]["level_ms"]))]
        kern = {k: round(sum(s["kernels"][k]["ms"] for s in sts) / n, 3) for k in sts[0]["kernels"]}
        dev = round(sum(s["ms_total"] for s in sts) / n, 3)
        out["orders"][order] = {"wall_ms_per_step": round(wall, 3), "device_ms": dev, "level_ms": levels,
                                "kernel_ms": kern}
        print(f"[relabel] {order}: wall {wall:.3f} ms, device {dev} ms, levels {levels}, kernels {kern}",
              file=sys.stderr, flush=True)
        snap.close()
        del g
    print(json.dumps(out))


if __name__ == "__main__":
    main()
