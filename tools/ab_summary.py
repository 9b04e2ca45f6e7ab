#!/usr/bin/env python3
"""Per-setting kernel times of a tools/ab_env.sh run: the last `--last` dispatches of each named kernel
(default: the last call of the command), in ms.

  python tools/ab_summary.py gpurun_out/ab_<tag> [--kernels a,b,c] [--last N]
"""
import csv
import os
import re
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    kern = None
    last = 1
    if "--kernels" in sys.argv:
        kern = sys.argv[sys.argv.index("--kernels") + 1].split(",")
    if "--last" in sys.argv:
        last = int(sys.argv[sys.argv.index("--last") + 1])
    for line in open(os.path.join(d, "settings.txt")):
        k, _, setting = line.strip().partition(" ")
        p = os.path.join(d, k, "run_kernel_trace.csv")
        if not os.path.exists(p):
            print(k, setting, "(no trace)")
            continue
        rows = sorted(csv.DictReader(open(p)), key=lambda r: int(r["Start_Timestamp"]))
        per = defaultdict(list)
        for r in rows:
            m = re.search(r"(hgx_[A-Za-z0-9_]+|k_[A-Za-z0-9_]+)", r["Kernel_Name"])
            n = m.group(1) if m else r["Kernel_Name"][:40]
            per[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
        names = kern or sorted(per, key=lambda n: -sum(per[n][-last:]))[:8]
        print(f"[{k}] {setting or '(default)'}: " + ", ".join(f"{n} {sum(per[n][-last:]):.3f}" for n in names if n in per))


if __name__ == "__main__":
    main()
