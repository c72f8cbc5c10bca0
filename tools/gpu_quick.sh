#!/bin/bash
# One GPU call: the pyramid / SIFT parity subset, then a rocprofv3 kernel profile of bench.py
# and the per-step kernel table (tools/kstats_step.py).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stages.py -m gpu -q -x --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_quick.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_quick.txt
[ $rc -ne 0 ] && exit $rc
rm -rf gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/prof.log | head -1
[ $rc -ne 0 ] && exit $rc
python3 tools/kstats_step.py gpurun_out/prof/run_kernel_stats.csv plan_device 4
