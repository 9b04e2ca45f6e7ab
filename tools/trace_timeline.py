#!/usr/bin/env python3
"""Timeline of the end of a rocprofv3 trace: kernels (per stream) and, when the run had --hip-trace,
the host's HIP API calls, in microseconds from the first kernel of the window.

  rocprofv3 --kernel-trace --hip-trace -f csv -d OUT -o run -- python3 tools/c5_step.py ...
  python tools/trace_timeline.py OUT [--last-us 2500] [--api-min-us 2]
"""
import argparse
import csv
import glob
import os


def rows(path):
    with open(path, newline="") as f:
        yield from csv.DictReader(f)


def short(name, n=44):
    name = name.split("(")[0]
    for p in ("void ", "hgx::"):
        name = name.replace(p, "")
    return name[:n]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last-us", type=float, default=2500.0)
    ap.add_argument("--api-min-us", type=float, default=2.0)
    args = ap.parse_args()
    kt = glob.glob(os.path.join(args.dir, "**", "*kernel_trace.csv"), recursive=True)
    at = glob.glob(os.path.join(args.dir, "**", "*hip_api_trace.csv"), recursive=True)
    ev = []
    for p in kt:
        for r in rows(p):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K s" + r.get("Stream_Id", "?"),
                       short(r["Kernel_Name"])))
    kend = max(e[1] for e in ev)
    t0 = kend - args.last_us * 1e3
    for p in at:
        for r in rows(p):
            b, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if (e - b) / 1e3 >= args.api_min_us:
                ev.append((b, e, "H t" + r.get("Thread_Id", "?")[-3:], r.get("Function", r.get("Operation", "?"))))
    win = sorted(e for e in ev if e[0] >= t0 and e[0] <= kend)
    first = min((e[0] for e in win if e[2].startswith("K")), default=t0)
    for b, e, who, name in win:
        print(f"{who:8s} {name:46s} {(b - first) / 1e3:9.1f} {(e - b) / 1e3:8.1f}")


if __name__ == "__main__":
    main()
