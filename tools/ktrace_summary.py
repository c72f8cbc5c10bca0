#!/usr/bin/env python3
"""Per (kernel, grid) average duration from a rocprofv3 --kernel-trace CSV, plus per-kernel
totals.  Usage: python tools/ktrace_summary.py <dir with *kernel_trace.csv> [runs]"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
runs = int(sys.argv[2]) if len(sys.argv) > 2 else 1
rows = []
for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
    rows += list(csv.DictReader(open(f)))
by = collections.defaultdict(list)
tot = collections.defaultdict(float)
for r in rows:
    k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
    k = k[5:] if k.startswith("void ") else k
    g = (int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    by[(k, g)].append(d)
    tot[k] += d
print(f"{'kernel':34s} {'total_us/run':>12s}")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"{k[:34]:34s} {v / runs:12.1f}")
print()
for (k, g), v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
    if sum(v) / runs < 5:
        continue
    print(f"{k[:34]:34s} {str(g):22s} n={len(v):4d} avg={sum(v) / len(v):8.2f} us")
