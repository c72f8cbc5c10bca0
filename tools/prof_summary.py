#!/usr/bin/env python3
"""Summarise a rocprofv3 .db (kernel trace): per-kernel count / total / avg, and one step's
launch sequence.  Usage: python tools/prof_summary.py gpurun_out/prof/run_results.db [steps]"""
import collections
import sqlite3
import sys

db = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else None
c = sqlite3.connect(db)
rows = c.execute("select name, duration, grid_x, grid_y, grid_z, workgroup_x, vgpr_count, "
                 "accum_vgpr_count, sgpr_count, lds_size, scratch_size from kernels order by start").fetchall()
agg = collections.OrderedDict()
for r in rows:
    name = r[0].split("(")[0].replace("(anonymous namespace)::", "")
    a = agg.setdefault(name, [0, 0.0, r[6], r[7], r[9], r[10]])
    a[0] += 1
    a[1] += r[1] / 1e3
tot = sum(v[1] for v in agg.values())
print(f"{'kernel':40s} {'calls':>6s} {'total_us':>10s} {'avg_us':>8s} {'%':>6s} vgpr agpr lds scratch")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{k[:40]:40s} {v[0]:6d} {v[1]:10.1f} {v[1] / v[0]:8.2f} {100 * v[1] / tot:6.1f} {v[2]} {v[3]} {v[4]} {v[5]}")
if steps:
    print(f"per step: {tot / steps:.1f} us of kernel time")
