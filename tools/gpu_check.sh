#!/bin/bash
# One GPU call: the given -m gpu test files (default: all), then a rocprofv3 kernel profile of
# bench.py and the per-step kernel table (tools/kstats_step.py).
#   TESTS="tests/test_gpu_stages.py" BENCH_ARGS="--workload synthetic" bash tools/gpu_check.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_check.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 5 gpurun_out/pytest_check.txt
[ $rc -ne 0 ] && exit $rc
[ -n "${NO_PROF:-}" ] && exit 0
rm -rf gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/prof.log | head -1
[ $rc -ne 0 ] && exit $rc
python3 tools/kstats_step.py gpurun_out/prof/run_kernel_stats.csv plan_device 4
