#!/bin/bash
# Round-5 iteration check in one GPU call: selected -m gpu tests (TESTS, default the parity +
# drop-in + stages files), then the one-step kernel timeline of parrington.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5check; rm -rf $O; mkdir -p $O
if [ -z "${NO_TESTS:-}" ]; then
  timeout -k 10 ${TLIM:-600} python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_dropin.py tests/test_gpu_stages.py} -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -n 3 $O/pytest.txt
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/steps -o run -- python3 tools/step_timeline.py > $O/steps.log 2>&1 || exit $?
python3 tools/timeline.py $O/steps/run_kernel_trace.csv --step 10 > $O/timeline_parrington.txt
tail -1 $O/timeline_parrington.txt
if [ -n "${BENCH:-}" ]; then
  timeout -k 10 300 python bench.py --no-cpu-baseline $BENCH > $O/bench.txt 2>&1 || exit $?
  tail -1 $O/bench.txt | cut -c1-300
fi
