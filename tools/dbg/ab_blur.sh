#!/bin/bash
# Kernel-trace stats of selected kernels (regex $KRE, default blur) for the working build and
# the tools/ab variants named in $VARIANTS.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for v in base ${VARIANTS}; do
  if [ $v = base ]; then L=""; else L=tools/ab/libpano_$v.so; fi
  PANO_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_$v -o run -- python3 tools/prof_features.py ${NRUN:-4} > gpurun_out/ab_$v.log 2>&1 || exit $?
  f=$(find gpurun_out/ab_$v -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$v" "${KRE:-blur}" <<'PY'
import csv, re, sys
f, v, kre = sys.argv[1:4]
tot = 0.0
for r in csv.DictReader(open(f)):
    if re.search(kre, r["Name"]):
        name = re.sub(r"\(anonymous namespace\)::", "", r["Name"]).split("(")[0]
        tot += float(r["TotalDurationNs"])
        print(f"{v:8s} {name[:44]:44s} n={r['Calls']:>4s} avg_us={float(r['AverageNs'])/1000:8.2f}")
print(f"{v:8s} TOTAL {tot/1000:.1f} us")
PY
done
