#!/bin/bash
# One GPU call: the JPEG decode tests first (new kernels, own time limit), then the round's
# tests / bench / rocprof (tools/gpu_round.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_jpeg.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_jpeg.txt 2>&1
rc=$?; echo "jpeg pytest rc=$rc"; tail -n 15 gpurun_out/pytest_jpeg.txt
[ $rc -gt 1 ] && exit $rc
[ "${JPEG_ONLY:-0}" = 1 ] && exit $rc
bash tools/gpu_round.sh
