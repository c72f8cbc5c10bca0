#!/bin/bash
# One GPU call: the headline bench (parrington, N=1) and the config-5 lines (synthetic 1080p
# weak: 19 frames; strong: the whole 144-frame / 143-pair batch at N=1, the denominator of
# the strong-scaling curve).  JSON lines in gpurun_out/bench_*.txt.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_parrington.txt 2>&1 || exit $?
tail -1 gpurun_out/bench_parrington.txt | cut -c1-400
timeout -k 10 600 python bench.py --workload synthetic --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_synthetic.txt 2>&1 || exit $?
tail -1 gpurun_out/bench_synthetic.txt | cut -c1-400
if [ "${STRONG:-1}" = 1 ]; then
  timeout -k 10 900 python bench.py --workload synthetic --scaling strong --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_synthetic_strong.txt 2>&1 || exit $?
  tail -1 gpurun_out/bench_synthetic_strong.txt | cut -c1-400
fi
