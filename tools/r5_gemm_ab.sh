#!/bin/bash
# dist_i8 / descriptor / orientation / extrema / tail kernel times per library variant (tools/ab/libpano_<v>.so, "base" = the tree's):
# rocprofv3 kernel stats of a short eager bench, the dist_i8 average per variant.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/gemm_ab; rm -rf $O; mkdir -p $O
for v in ${VARIANTS:-base abl1 abl2 nostag w2}; do
  lib=""; [ "$v" != base ] && lib=tools/ab/libpano_$v.so
  PANO_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 bench.py --workload ${WORK:-synthetic} --steps 3 --warmup 1 --no-cpu-baseline > $O/$v.log 2>&1 || { tail -3 $O/$v.log; exit 1; }
  python3 - "$O/$v/run_kernel_stats.csv" "$v" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    if any(k in r["Name"] for k in ("dist_i8", "descriptor_wave", "orientation", "extrema_stream", "blur_tail")):
        print(sys.argv[2], r["Name"][:40], "calls", r["Calls"], "avg_us", round(float(r["AverageNs"]) / 1e3, 1))
PY
  rm -rf $O/$v
done
