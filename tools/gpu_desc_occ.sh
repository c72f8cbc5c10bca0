#!/bin/bash
# Descriptor register-budget selection: GPU tests with the default selection and with the
# large-batch instance forced (PANO_DESC_BIG_MIN=1), then one bench line per workload.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/descocc
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 $O/pytest.txt
[ $rc -ne 0 ] && exit $rc
PANO_DESC_BIG_MIN=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stages.py -m gpu -q -x --timeout 300 --timeout-method thread -k "sift or 1080p or 2047 or descriptors or gui" > $O/pytest_big.txt 2>&1
rc=$?; echo "pytest big rc=$rc"; tail -n 2 $O/pytest_big.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --steps 40 --warmup 3 --no-cpu-baseline > $O/bench_p.txt 2>&1 || exit $?
echo "parrington $(grep -o '"ms_per_step": [0-9.]*' $O/bench_p.txt | head -1) $(grep -o '"descriptor": [0-9.]*' $O/bench_p.txt | head -1)"
timeout -k 10 300 python3 bench.py --workload synthetic --steps 8 --warmup 2 --no-cpu-baseline > $O/bench_s.txt 2>&1 || exit $?
echo "synthetic $(grep -o '"ms_per_step": [0-9.]*' $O/bench_s.txt | head -1) $(grep -o '"descriptor": [0-9.]*' $O/bench_s.txt | head -1)"
exit 0
