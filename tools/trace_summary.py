#!/usr/bin/env python3
"""Per-kernel totals from a rocprofv3 --kernel-trace CSV (…_kernel_trace.csv).

    python tools/trace_summary.py gpurun_out/prof/run_kernel_trace.csv [--shapes]
"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    n = re.sub(r"^void ", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).split("(")[0]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    agg[n].append((d, r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"]))
tot = sum(x[0] for v in agg.values() for x in v)
print(f"{'kernel':50s} {'calls':>6s} {'total_us':>10s} {'avg_us':>8s} {'%':>6s}")
for n, v in sorted(agg.items(), key=lambda kv: -sum(x[0] for x in kv[1])):
    t = sum(x[0] for x in v)
    print(f"{n[:50]:50s} {len(v):6d} {t:10.1f} {t / len(v):8.2f} {100 * t / tot:6.1f}")
if "--shapes" in sys.argv:
    b = collections.defaultdict(list)
    for n, v in agg.items():
        for x in v:
            b[(n, x[1], x[2], x[3])].append(x[0])
    for k in sorted(b, key=lambda k: -sum(b[k]))[:30]:
        print(k, len(b[k]), round(sum(b[k]) / len(b[k]), 2))
