#!/bin/bash
# Kernel-trace timings (per kernel and grid) of kernels matching $KRE (default blur) for the
# working build and the tools/ab variants named in $VARIANTS.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for v in base ${VARIANTS}; do
  if [ $v = base ]; then L=""; else L=tools/ab/libpano_$v.so; fi
  PANO_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ab_$v -o run -- python3 tools/prof_features.py ${NRUN:-4} > gpurun_out/ab_$v.log 2>&1 || exit $?
  f=$(find gpurun_out/ab_$v -name "*kernel_trace.csv" | head -1)
  python3 tools/dbg/trace_groups.py "$f" "$v" "${KRE:-blur}" ${NRUN:-4}
done
