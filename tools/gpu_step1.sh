#!/bin/bash
# First GPU check of the f32 (OpenCV 4.x) blur and the sift_impl stage functions.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  "tests/test_gpu_parity.py::test_pyramid_bit_exact" tests/test_gpu_stages.py > gpurun_out/t1.log 2>&1
rc=$?
tail -40 gpurun_out/t1.log
exit $rc
