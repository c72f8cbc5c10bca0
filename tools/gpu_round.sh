#!/bin/bash
# One GPU call: gpu tests, bench, rocprofv3 kernel stats.  Stops after any crash-class exit.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) [ "$1" -gt 128 ] && return 0; return 1;; esac; }
STEPS=${STEPS:-20}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.txt 2>&1
  rc=$?; echo "pytest rc=$rc" | tee -a gpurun_out/pytest_gpu.txt; tail -n 5 gpurun_out/pytest_gpu.txt
  # any failing GPU test may be a device fault: run nothing more on the GPU in this call
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 600 python bench.py --steps $STEPS --warmup 3 ${BENCH_ARGS:-} > gpurun_out/bench.txt 2>&1
rc=$?; echo "bench rc=$rc"; tail -n 3 gpurun_out/bench.txt
[ $rc -ne 0 ] && exit $rc
if [ "${SKIP_PROF:-0}" != 1 ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"
  find gpurun_out/prof -name "*stats*" | head
fi
