"""Average duration per (kernel, grid) from a rocprofv3 kernel_trace.csv, plus per-run total."""
import csv
import re
import sys
from collections import defaultdict

f, tag, kre, nrun = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
g = defaultdict(list)
for r in csv.DictReader(open(f)):
    if not re.search(kre, r["Kernel_Name"]):
        continue
    name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"]).split("(")[0].replace("void ", "")
    key = (name, r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
    g[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
tot = 0.0
for k, v in sorted(g.items(), key=lambda kv: -sum(kv[1])):
    tot += sum(v)
    print(f"{tag:8s} {k[0][:34]:34s} grid={k[1]}x{k[2]}x{k[3]:<4s} n={len(v):3d} avg_us={sum(v)/len(v):8.2f}")
print(f"{tag:8s} TOTAL per run {tot/nrun:.1f} us")
