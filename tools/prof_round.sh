#!/bin/bash
# One GPU call: kernel-trace + stats profile of bench.py (parrington, graph replay) and the
# one-step timeline (tools/timeline.py) -> gpurun_out/prof_<tag>/
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-cur}
D=gpurun_out/prof_$TAG
rm -rf $D && mkdir -p $D
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > $D/log.txt 2>&1 || exit $?
K=$(find $D -name "*kernel_trace.csv" | head -1)
python3 tools/timeline.py $K --step -3 > $D/timeline.txt && tail -60 $D/timeline.txt
