#!/bin/bash
# Round-end evidence in one call: every -m gpu test, smoke(), then tools/refresh_profiles.sh.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_gpu.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 2 gpurun_out/smoke.txt
[ $rc -ne 0 ] && exit $rc
bash tools/refresh_profiles.sh
