#!/bin/bash
# One GPU call: gpu tests, bench, rocprofv3 kernel stats.  Stops after any crash-class exit
# (timeout 124/137, abort 134, segfault 139, any signal > 128); plain test failures (rc 1)
# let the bench run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=${STEPS:-20}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.txt 2>&1
  rc=$?; echo "pytest rc=$rc" | tee -a gpurun_out/pytest_gpu.txt; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.txt | tail -n 30
  [ $rc -gt 1 ] && exit $rc
fi
timeout -k 10 600 python bench.py --steps $STEPS --warmup 3 ${BENCH_ARGS:-} > gpurun_out/bench.txt 2>&1
rc=$?; echo "bench rc=$rc"; tail -n 3 gpurun_out/bench.txt | cut -c1-3000
[ $rc -ne 0 ] && exit $rc
if [ "${SKIP_PROF:-0}" != 1 ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"
  find gpurun_out/prof -name "*stats*" | head
fi
exit 0
