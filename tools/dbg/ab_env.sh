#!/bin/bash
# Kernel-trace timings of kernels matching $KRE under each environment setting in $ENVS
# (space-separated list of VAR=value[,VAR=value] items; "base" = unchanged environment).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for e in ${ENVS:-base}; do
  tag=$(echo "$e" | tr ',=' '__')
  ( [ "$e" != base ] && for kv in ${e//,/ }; do export "$kv"; done
    timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/abe_$tag -o run -- python3 tools/prof_features.py ${NRUN:-4} > gpurun_out/abe_$tag.log 2>&1 ) || exit $?
  f=$(find gpurun_out/abe_$tag -name "*kernel_trace.csv" | head -1)
  python3 tools/dbg/trace_groups.py "$f" "$tag" "${KRE:-blur}" ${NRUN:-4}
done
