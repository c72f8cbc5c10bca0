#!/usr/bin/env python3
"""Timeline of one stitch step from a rocprofv3 --kernel-trace CSV: every kernel of the
chosen step with its start offset, duration and the idle gap before it (what is on the
critical path, what overlaps).

    python tools/timeline.py gpurun_out/prof/run_kernel_trace.csv [--first gray_frames] [--step -2]

A step starts at each launch of the --first kernel (default gray_frames); --step picks one
(negative = from the end; default the second last, so the trace's tail does not cut it).
"""
import argparse
import csv
import re

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--first", default="gray_frames")
ap.add_argument("--step", type=int, default=-2)
a = ap.parse_args()

rows = []
for r in csv.DictReader(open(a.csv)):
    n = re.sub(r"^void ", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).split("(")[0]
    n = re.sub(r"\s+", "", n)
    g = (r.get("Grid_Size_X", ""), r.get("Grid_Size_Y", ""), r.get("Grid_Size_Z", ""))
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n, g))
rows.sort()
starts = [i for i, r in enumerate(rows) if r[2].startswith(a.first)]
i0 = starts[a.step]
i1 = starts[a.step + 1] if a.step + 1 < 0 or a.step + 1 < len(starts) else len(rows)
if a.step == -1:
    i1 = len(rows)
step = rows[i0:i1]
t0 = step[0][0]
busy_end = t0
print(f"{'start_us':>9s} {'dur_us':>8s} {'gap_us':>7s}  kernel  grid")
for s, e, n, g in step:
    gap = (s - busy_end) / 1e3
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {gap:7.1f}  {n[:60]}  {'x'.join(g)}")
    busy_end = max(busy_end, e)
# busy = the union of the kernels' intervals (overlapping side-stream kernels counted once);
# the step span runs to the next step's first kernel, so the host gap between steps counts
nxt = rows[i1][0] if i1 < len(rows) else busy_end
busy, cur = 0, t0
for s, e, _, _ in step:
    s = max(s, cur)
    if e > s:
        busy += e - s
        cur = e
print(f"step span {(busy_end - t0) / 1e3:.1f} us to the last kernel's end, {(nxt - t0) / 1e3:.1f} us to the next "
      f"step; GPU busy {busy / 1e3:.1f} us; idle {(nxt - t0 - busy) / 1e3:.1f} us; {len(step)} kernels")
