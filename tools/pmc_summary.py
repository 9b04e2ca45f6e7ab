#!/usr/bin/env python3
"""Summarise a tools/profile_round.sh output directory into profiles/.

  python tools/pmc_summary.py gpurun_out/prof_<tag> <tag> [workload] [--until KERNEL]

--until KERNEL keeps only the dispatches before the first launch of a kernel whose name contains
KERNEL after the first BFS gather (bench.py runs config 2 first, then builds the config-3 snapshot:
`--until k_validate` isolates the config-2 leg of the default bench command).
--from-last KERNEL keeps only the dispatches from the last launch of KERNEL on (the last call of a tool
that repeats one call: `--from-last hgx_ls_seed` is the steady-state drop-in call of tools/seq_c2.py).
--from KERNEL keeps only the dispatches from the first launch of KERNEL after the first BFS gather on
(`--from k_validate` with `--no-queries`: the config-4 leg, whose snapshot is built after the config-2 leg).
--min-ms X drops every dispatch shorter than X ms (by the trace pass; tools/seq_c5.py's single-seed calls
beside its batched ones).

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
import subprocess
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


def cutoff(rows, until, after="hgx_link_gather"):
    """Dispatch id of the first launch of `until` that follows a launch of `after` (None = keep
    everything)."""
    if not until:
        return None
    first = [int(r["Dispatch_Id"]) for r in rows if after in r["Kernel_Name"]]
    if not first:
        return None
    ids = [int(r["Dispatch_Id"]) for r in rows if until in r["Kernel_Name"] and int(r["Dispatch_Id"]) > min(first)]
    return min(ids) if ids else None


def first_kept(rows, from_last):
    """Dispatch id of the last launch of `from_last` (None = keep everything)."""
    if not from_last:
        return None
    ids = [int(r["Dispatch_Id"]) for r in rows if from_last in r["Kernel_Name"]]
    return max(ids) if ids else None


def load_counter(path, counter, until=None, from_last=None, from_first=None):
    acc = defaultdict(list)
    if not os.path.exists(path):
        return acc
    with open(path) as f:
        rows = list(csv.DictReader(f))
    cut = cutoff(rows, until)
    lo = first_kept(rows, from_last) if from_last else cutoff(rows, from_first)
    for row in rows:
        if lo is not None and int(row["Dispatch_Id"]) < lo:
            continue
        if row["Counter_Name"] == counter and (cut is None or int(row["Dispatch_Id"]) < cut):
            acc[short(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    return acc


def load_trace(path, until=None, from_last=None, from_first=None):
    acc = defaultdict(list)
    with open(path) as f:
        rows = list(csv.DictReader(f))
    cut = cutoff(rows, until)
    lo = first_kept(rows, from_last) if from_last else cutoff(rows, from_first)
    for row in rows:
        if lo is not None and int(row["Dispatch_Id"]) < lo:
            continue
        if cut is None or int(row["Dispatch_Id"]) < cut:
            acc[short(row["Kernel_Name"])].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6)
    return acc


def main():
    argv = sys.argv[1:]
    until = from_last = from_first = None
    if "--until" in argv:
        k = argv.index("--until")
        until = argv[k + 1]
        del argv[k:k + 2]
    min_ms = 0.0
    if "--min-ms" in argv:
        k = argv.index("--min-ms")
        min_ms = float(argv[k + 1])
        del argv[k:k + 2]
    if "--from" in argv:
        k = argv.index("--from")
        from_first = argv[k + 1]
        del argv[k:k + 2]
    if "--from-last" in argv:
        k = argv.index("--from-last")
        from_last = argv[k + 1]
        del argv[k:k + 2]
    d, tag = argv[0], argv[1]
    workload = argv[2] if len(argv) > 2 else "config2"
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prof = os.path.join(root, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = os.path.join(d, "trace", "run_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(prof, f"{tag}_kernel_stats.csv"))
    trace = load_trace(os.path.join(d, "trace", "run_kernel_trace.csv"), until, from_last, from_first)
    if min_ms > 0:   # the passes dispatch in the same order: drop the short launches' counter values by rank
        with open(os.path.join(d, "trace", "run_kernel_trace.csv")) as f:
            rows = sorted(csv.DictReader(f), key=lambda r: int(r["Dispatch_Id"]))
        short_rank = defaultdict(set)
        seen = defaultdict(int)
        for r in rows:
            k = short(r["Kernel_Name"])
            if (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 < min_ms:
                short_rank[k].add(seen[k])
            seen[k] += 1
        trace = {k: [t for t in v if t >= min_ms] for k, v in trace.items()}
        trace = {k: v for k, v in trace.items() if v}
    fetch = load_counter(os.path.join(d, "fetch", "run_counter_collection.csv"), "FETCH_SIZE", until, from_last, from_first)
    write = load_counter(os.path.join(d, "write", "run_counter_collection.csv"), "WRITE_SIZE", until, from_last, from_first)
    if min_ms > 0:
        fetch = {k: [v for i, v in enumerate(vs) if i not in short_rank[k]] for k, vs in fetch.items()}
        write = {k: [v for i, v in enumerate(vs) if i not in short_rank[k]] for k, vs in write.items()}
    # the commit of the code the passes measured (this script runs in the repository right after the
    # gpurun call that took them); bench.py copies it into the line's traffic_from, so the provenance
    # survives a GPU lease without .git
    try:
        commit = subprocess.run(["git", "-C", root, "rev-parse", "--short=12", "HEAD"], capture_output=True,
                                text=True, timeout=10).stdout.strip() or None
        dirty = bool(subprocess.run(["git", "-C", root, "status", "--porcelain", "--untracked-files=no", "--",
                                     "hypergraphdb_amd", "include"], capture_output=True, text=True,
                                    timeout=10).stdout.strip())
    except Exception:
        commit, dirty = None, None
    rows, js = [], {"tag": tag, "workload": workload, "kernels": {}, "commit": commit, "from_last": from_last,
                    "from": from_first,
                    "min_ms": min_ms or None,
                    "commit_dirty": dirty,
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
        if until:
            f.write(f"Dispatches before the first `{until}` launch after the BFS only (the {workload} leg of the command).\n\n")
        if from_last:
            f.write(f"Dispatches from the last `{from_last}` launch on only (the command's last call).\n\n")
        if from_first:
            f.write(f"Dispatches from the first `{from_first}` launch after the BFS on only (the {workload} leg).\n\n")
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
