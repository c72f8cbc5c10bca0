#!/bin/bash
# Kernel-trace profile of N parrington stitches (tools/prof_features.py) -> per-kernel summary.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
N=${N:-5}
rm -rf gpurun_out/kt && mkdir -p gpurun_out/kt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt -o run -- python3 tools/prof_features.py $N > gpurun_out/kt/log.txt 2>&1 || exit $?
python tools/ktrace_summary.py gpurun_out/kt $N > gpurun_out/kt/summary.txt && cat gpurun_out/kt/summary.txt
