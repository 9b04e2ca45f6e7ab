#!/usr/bin/env python3
"""Partitioned-BFS rehearsal on ONE GPU: config 4 (scaled) split into NP vertex-cut parts, all on
cuda:0, run as one in-process group with the parts' device work serialised (HGX_OPT_PART_SERIAL),
so each part's kernel times are those it would have alone on its own GPU.

Per level it reports, over the parts: the largest per-part device time (local expansion + pack /
apply kernels of the exchange), the bytes each part ships, and the largest bytes one part sends to
ONE peer (an all-to-all over xGMI runs its 7 peer links in parallel, each at ~153 GB/s:
MI355X_MICROARCH / SURVEY.md 5).  The modelled NP-GPU level time is
    max_p device_ms(p) + max_pair_bytes / 153 GB/s + host round trips x --sync-us
(no overlap of exchange and compute assumed), summed over the levels; the 1-part run is the
replica on one GPU.  Host round trips of a level: what the engine counted (stats level_xtrips:
the count and statistics read-backs and the count / termination all-gathers -- 6 with counted
records in both phases, 4 with a static broadcast or at the final level of a depth-limited
traversal, which has no broadcast phase; the all-to-alls are ordered on the stream without a host
wait); --sync-us prices one (a small RCCL collective or a read-back at 8 ranks, default 40 us).
Counts of every source must equal the replica's.

  python tools/bench_part.py --scale 0.25 --parts 1 8 --out gpurun_out/part.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

XGMI_LINK_GBS = 153.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=0.25)
    ap.add_argument("--parts", type=int, nargs="+", default=[1, 8])
    ap.add_argument("--sources", type=int, default=1024)
    ap.add_argument("--depth", type=int, default=4)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--out", default="")
    ap.add_argument("--sync-us", type=float, default=40.0, help="price of one host round trip of the exchange")
    ap.add_argument("--xmode", type=int, nargs="+", default=[0],
                    help="HGX_OPT_PART_EXCHANGE values to measure at NP > 1 (0 / 1 records; the static slots (2) were removed)")
    args = ap.parse_args()
    from hypergraphdb_amd import _lib, synth
    from hypergraphdb_amd.partition import Shard, ShardSnapshot, partition_plan, pbfs_batch_group
    t0 = time.time()
    g = synth.config4(scale=args.scale, n_sources=args.sources)
    print(f"config4 x{args.scale}: A={g['num_atoms']} P={len(g['tgt_idx'])} in {time.time() - t0:.1f}s", flush=True)
    rows = []
    state = {"ref_counts": None, "ref_ms": None}
    for NP in args.parts:
        t0 = time.time()
        plan = partition_plan(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"], NP)
        plan_s = time.time() - t0
        snaps, info = [], []
        for p in range(NP):
            sh = Shard.build(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"], NP, p, plan)
            info.append({"local_atoms": sh.n_local, "owned_atoms": sh.n_owned, "local_links": sh.n_links,
                         "local_pins": sh.n_pins})
            snaps.append(ShardSnapshot(sh, 0))
            sh.close()
            snaps[-1].set_timing(True)
            if NP > 1:
                snaps[-1].set_serial(True)
        build_s = time.time() - t0
        print(f"{NP} parts: plan {plan_s:.1f}s, built in {build_s:.1f}s", flush=True)
        for xmode in (args.xmode if NP > 1 else [0]):
            for sn in snaps:
                if NP > 1:
                    sn.set_option(_lib.HGX_OPT_PART_EXCHANGE, xmode)
            measure(args, g, snaps, NP, xmode, plan_s, build_s, info, rows, state)
        for s in snaps:
            s.close()
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"scale": args.scale, "sources": args.sources, "depth": args.depth,
                       "xgmi_link_GBps": XGMI_LINK_GBS, "host_sync_us": args.sync_us, "rows": rows}, f, indent=1)


def measure(args, g, snaps, NP, xmode, plan_s, build_s, info, rows, state):
    from hypergraphdb_amd.partition import pbfs_batch_group
    if True:
        r = pbfs_batch_group(snaps, g["seeds"], args.depth)
        counts = r.counts()
        st0 = r.stats(accounting=True)
        r.close()
        if state["ref_counts"] is None:
            state["ref_counts"] = counts
        assert np.array_equal(counts, state["ref_counts"]), f"{NP} parts (xmode {xmode}) differ from {args.parts[0]}"
        ref_ms = state["ref_ms"]
        sts = []
        for _ in range(args.steps):
            r = pbfs_batch_group(snaps, g["seeds"], args.depth)
            sts.append(r.stats(accounting=False))
            r.close()
        nlev = max(len(s[p]["level_ms"]) for s in sts for p in range(NP))
        levels = []
        for d in range(nlev):
            def avg(key, p):
                v = [s[p][key][d] for s in sts if d < len(s[p][key])]
                return sum(v) / max(len(v), 1)
            dev = [avg("level_ms", p) for p in range(NP)]
            xms = [avg("level_xms", p) for p in range(NP)]
            xb = [avg("level_xbytes", p) for p in range(NP)]
            pm = max(max((s[p]["level_xpair_max"][d] for s in sts if d < len(s[p]["level_xpair_max"])), default=0)
                     for p in range(NP))
            link_ms = pm / (XGMI_LINK_GBS * 1e9) * 1e3
            # the level's host round trips as the engine counted them (count / statistics read-backs and
            # count all-gathers: 6 with counted records in both phases, 4 with a static broadcast or on
            # the final level of a depth-limited traversal, which has no broadcast phase)
            trips = max((s[p].get("level_xtrips", [0] * nlev)[d] for s in sts for p in range(NP)
                         if d < len(s[p].get("level_xtrips", []))), default=0)
            sync_ms = (trips * args.sync_us / 1e3) if NP > 1 else 0.0
            levels.append({"max_part_device_ms": round(max(dev), 3), "max_part_exchange_kernels_ms": round(max(xms), 3),
                           "host_trips": trips,
                           "bytes_per_part_max": max(xb), "max_pair_bytes": pm, "max_pair_link_ms": round(link_ms, 3),
                           "host_sync_ms": round(sync_ms, 3),
                           "model_level_ms": round(max(dev) + link_ms + sync_ms, 3),
                           "exchange_below_compute": link_ms < max(dev) - max(xms)})
        model_ms = sum(lv["model_level_ms"] for lv in levels)
        per = []
        for p in range(NP):
            ss = [s[p] for s in sts]
            # kernel time of the part (its levels' kernel events; in serial mode the part's stream also
            # idles while the other parts run, so ms_total would count their time too)
            per.append({"device_ms": round(sum(sum(s["level_ms"]) for s in ss) / len(ss), 3),
                        "span_ms": round(sum(s["ms_total"] for s in ss) / len(ss), 3),
                        "kernel_ms": {k: round(sum(s["kernels"][k]["ms"] for s in ss) / len(ss), 3)
                                      for k in ss[0]["kernels"]},
                        "exchange_kernels_ms": round(sum(s["ms_exchange"] for s in ss) / len(ss), 3),
                        "bytes_exchanged": sum(s["bytes_exchanged"] for s in ss) / len(ss),
                        "nonzero_word_frac": (ss[0]["xwords_nonzero"] / ss[0]["xwords_total"]
                                              if ss[0]["xwords_total"] else None),
                        "traversed_edges": st0[p]["traversed_edges"], **info[p]})
        if NP == 1:
            ref_ms = state["ref_ms"] = per[0]["device_ms"]
        row = {"parts": NP, "xmode": xmode, "plan_s": round(plan_s, 1), "build_s": round(build_s, 1),
               "traversed_edges": sum(x["traversed_edges"] for x in per),
               "max_part_device_ms": round(max(x["device_ms"] for x in per), 3),
               "model_step_ms": round(model_ms, 3),
               "model_speedup_vs_1_part": round(ref_ms / model_ms, 3) if ref_ms and NP > 1 else None,
               "device_ms_vs_1_part": round(ref_ms / max(x["device_ms"] for x in per), 3) if ref_ms and NP > 1 else None,
               "exchange_bytes_total": sum(x["bytes_exchanged"] for x in per), "levels": levels, "per_part": per}
        rows.append(row)
        print(json.dumps({k: v for k, v in row.items() if k not in ("per_part",)}), flush=True)


if __name__ == "__main__":
    main()
