#!/usr/bin/env python3
"""Per-step timeline of a rocprofv3 kernel trace of bench.py (graph replay): the fastest
step's kernels with start/end offsets, GPU-busy time and the gap to the next step.
Usage: python tools/graph_trace.py <trace dir> [first_kernel_substring]"""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
first = sys.argv[2] if len(sys.argv) > 2 else "cyl_scatter"
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
nm = lambda r: r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[:34]
idx = [i for i, r in enumerate(rows) if first in nm(r)]
best = None
for a, b in zip(idx[:-1], idx[1:]):
    gap = int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])
    if best is None or gap < best[0]:
        best = (gap, a, b)
gap, a, b = best
t0 = int(rows[a]["Start_Timestamp"])
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows[a:b])
busy, (cs, ce) = 0, iv[0]
for s, e in iv[1:]:
    if s > ce:
        busy += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
busy += ce - cs
last_end = max(e for _, e in iv)
print(f"steps seen {len(idx)}; fastest step period {gap / 1e3:.1f} us, GPU busy {busy / 1e3:.1f} us, "
      f"host gap after last kernel {(int(rows[b]['Start_Timestamp']) - last_end) / 1e3:.1f} us")
for r in rows[a:b]:
    s = (int(r["Start_Timestamp"]) - t0) / 1e3
    e = (int(r["End_Timestamp"]) - t0) / 1e3
    print(f"{s:8.1f} {e:8.1f} {e - s:7.1f}  q{r['Queue_Id']}  {nm(r)}  {r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}")
