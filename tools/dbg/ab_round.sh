#!/bin/bash
# One GPU call: gpu parity tests of the working tree, then bench.py kernel-class A/B of the
# working tree against tools/ab variants ($VARIANTS) on parrington and (AB_SYN=1) synthetic 1080p.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.txt 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -n 15 gpurun_out/pytest_gpu.txt
  [ $rc -ne 0 ] && exit $rc
fi
BENCH_ARGS="--steps 10 --warmup 2" bash tools/dbg/ab_bench.sh || exit $?
if [ "${AB_SYN:-0}" = 1 ]; then
  for v in base ${VARIANTS}; do
    L=""; E=""
    case $v in base) ;; env:*) E=${v#env:} ;; *) L=tools/ab/libpano_$v.so ;; esac
    env $E PANO_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --workload synthetic --steps 4 --warmup 1 > gpurun_out/abs_$v.txt 2>&1 || exit $?
    python3 -c "
import json;d=json.loads(open('gpurun_out/abs_$v.txt').read().strip().split('\n')[-1]);print('syn $v', d['ms_per_step'], json.dumps(d['kernels_ms_per_step']))"
  done
fi
