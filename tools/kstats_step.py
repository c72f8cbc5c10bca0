#!/usr/bin/env python3
"""Per-step kernel table from a rocprofv3 kernel_stats.csv: us per step for each kernel,
steps = the number of calls of a once-per-step kernel (default: plan_device)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
anchor = sys.argv[2] if len(sys.argv) > 2 else "plan_device"
steps = next((int(r["Calls"]) for r in rows if anchor in r["Name"]), 1)
tot = 0.0
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    n = r["Name"].replace("(anonymous namespace)::", "")
    t = float(r["TotalDurationNs"]) / steps / 1000
    tot += t
    if t >= float(sys.argv[3] if len(sys.argv) > 3 else 2.0):
        print(f"{t:8.1f} us/step  calls/step={int(r['Calls']) / steps:5.2f}  avg={float(r['AverageNs']) / 1000:7.1f}  {n[:100]}")
print(f"total {tot:.1f} us/step over {steps} steps")
