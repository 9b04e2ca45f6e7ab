#!/usr/bin/env python3
"""Summarise a tools/profile_round.sh output directory into profiles/.

  python tools/pmc_summary.py gpurun_out/prof_<tag> <tag> [workload]

Writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim)
  profiles/<tag>_summary.md         per-kernel launches / avg duration / PMC HBM bytes
  profiles/pmc_<workload>.json      per-kernel HBM bytes per launch (read by bench.py)

HBM bytes follow MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE are in KiB,
collected in separate passes; on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced
stream, so bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.  The FETCH_SIZE doubling is calibrated
for 16-B/lane streaming reads; for the gathers of this engine it is an upper estimate (noted).
"""
import csv
import json
import os
import re
import shutil
import sys
from collections import defaultdict


# kernels that implement one engine kind (HGX_K_* of include/hgx.h): the tile-staged dense kernels
# report under the kind's name so bench.py finds their PMC bytes
KIND = {"hgx_link_gather2": "hgx_link_gather", "hgx_atom_pull2": "hgx_atom_pull"}


def short(name):
    m = re.search(r"\b(hgx_[A-Za-z0-9_]+|k_[A-Za-z0-9_]+)\b", name)
    if m:
        return KIND.get(m.group(1), m.group(1))
    if "radix_sort" in name:
        return "rocprim_radix_sort"
    if "scan" in name:
        return "rocprim_scan"
    return name.split("(")[0][-60:]


def load_counter(path, counter):
    acc = defaultdict(list)
    if not os.path.exists(path):
        return acc
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == counter:
                acc[short(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    return acc


def load_trace(path):
    acc = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            acc[short(row["Kernel_Name"])].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6)
    return acc


def main():
    d, tag = sys.argv[1], sys.argv[2]
    workload = sys.argv[3] if len(sys.argv) > 3 else "config2"
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prof = os.path.join(root, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = os.path.join(d, "trace", "run_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(prof, f"{tag}_kernel_stats.csv"))
    trace = load_trace(os.path.join(d, "trace", "run_kernel_trace.csv"))
    fetch = load_counter(os.path.join(d, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = load_counter(os.path.join(d, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    rows, js = [], {"tag": tag, "workload": workload, "kernels": {},
                    "note": "bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024 per launch (gfx950 FETCH_SIZE correction)"}
    for k in sorted(trace, key=lambda k: -sum(trace[k])):
        t = trace[k]
        f = fetch.get(k, [])
        w = write.get(k, [])
        fb = 2.0 * 1024 * sum(f) / len(f) if f else None
        wb = 1024 * sum(w) / len(w) if w else None
        hbm = (fb or 0) + (wb or 0) if (f or w) else None
        avg = sum(t) / len(t)
        rows.append((k, len(t), sum(t), avg, fb, wb, hbm))
        js["kernels"][k] = {"launches": len(t), "avg_ms": avg, "fetch_bytes_per_launch": fb,
                            "write_bytes_per_launch": wb, "hbm_bytes_per_launch": hbm,
                            "hbm_GBps": (hbm / (avg / 1e3) / 1e9) if hbm else None}
    with open(os.path.join(prof, f"pmc_{workload}.json"), "w") as f:
        json.dump(js, f, indent=1)
    with open(os.path.join(prof, f"{tag}_summary.md"), "w") as f:
        f.write(f"# rocprofv3 summary {tag} ({workload})\n\n")
        f.write("Kernel trace: `rocprofv3 --kernel-trace --stats`; HBM bytes from separate `--pmc FETCH_SIZE` and\n"
                "`--pmc WRITE_SIZE` passes, bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 per launch.\n\n")
        f.write("| kernel | launches | total ms | avg ms | fetch B/launch | write B/launch | HBM GB/s |\n")
        f.write("|---|---|---|---|---|---|---|\n")
        for k, n, tot, avg, fb, wb, hbm in rows:
            gbs = f"{hbm / (avg / 1e3) / 1e9:.0f}" if hbm else "-"
            f.write(f"| {k} | {n} | {tot:.2f} | {avg:.4f} | {fb or 0:.3e} | {wb or 0:.3e} | {gbs} |\n")
    print(open(os.path.join(prof, f"{tag}_summary.md")).read())


if __name__ == "__main__":
    main()
