#!/bin/bash
# The drop-in stage-function tests (sift_impl.py stage functions through libpano) + drop-in tests.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 500 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_dropin.py -m gpu -v -x --timeout 300 --timeout-method thread > gpurun_out/t_stages.txt 2>&1
echo "tests rc=$?"; grep -E "PASS|FAIL|Error|assert" gpurun_out/t_stages.txt | tail -40
