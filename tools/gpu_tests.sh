#!/bin/bash
# Selected -m gpu test files in one process (default: all), output to gpurun_out/pytest_sel.txt.
#   TESTS="tests/test_jpeg.py tests/test_gpu_stages.py" bash tools/gpu_tests.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 ${TLIM:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_sel.txt 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_sel.txt | tail -n 3
exit $rc
