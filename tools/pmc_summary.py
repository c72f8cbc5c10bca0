#!/usr/bin/env python3
"""Aggregate rocprofv3 counter_collection CSVs per kernel (mean over dispatches).
Usage: python tools/pmc_summary.py gpurun_out/pmc"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        if k.startswith("void "):
            k = k[5:]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in sorted(glob.glob(os.path.join(root, "p1", "*kernel_trace.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        if k.startswith("void "):
            k = k[5:]
        dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, cs in sorted(agg.items()):
    d = dur.get(k, [0])
    print(f"== {k}  dispatches={len(d)} avg_us={sum(d) / max(len(d), 1):.2f}")
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} {sum(v) / len(v):16.1f}")
