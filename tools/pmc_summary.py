#!/usr/bin/env python3
"""Aggregate rocprofv3 counter_collection CSVs per (kernel, grid size): mean over dispatches.
Usage: python tools/pmc_summary.py gpurun_out/pmc"""
import collections
import csv
import glob
import os
import sys


def kname(s):
    k = s.replace("(anonymous namespace)::", "").split("(")[0]
    return k[5:] if k.startswith("void ") else k


root = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        key = (kname(r["Kernel_Name"]), int(r["Grid_Size"]))
        agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if f.endswith(os.path.join("p1", os.path.basename(f))) and r["Counter_Name"] == "SQ_WAVES":
            dur[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for key, cs in sorted(agg.items(), key=lambda kv: (kv[0][0], -kv[0][1])):
    d = dur.get(key, [0])
    print(f"== {key[0]} grid={key[1]}  dispatches={len(d)} avg_us={sum(d) / max(len(d), 1):.2f}")
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} {sum(v) / len(v):16.1f}")
