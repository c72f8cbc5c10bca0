#!/bin/bash
# Kernel-trace profile of N parrington stitches (tools/prof_features.py) -> per-kernel summary.
# KT=<dir> names the output directory (default gpurun_out/kt).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
N=${N:-5}
KT=${KT:-gpurun_out/kt}
rm -rf $KT && mkdir -p $KT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $KT -o run -- python3 tools/prof_features.py $N > $KT/log.txt 2>&1 || exit $?
python tools/ktrace_summary.py $KT $N > $KT/summary.txt && cat $KT/summary.txt
