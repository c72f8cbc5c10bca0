#!/bin/bash
# bench.py kernel-class times for the working build and the variants in $VARIANTS: a name is
# tools/ab/libpano_<name>.so, or env:VAR=value runs the working build with that environment
# (BENCH_ARGS passed through); one JSON summary line per variant.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in base ${VARIANTS}; do
  L=""; E=""
  case $v in base) ;; env:*) E=${v#env:} ;; *) L=tools/ab/libpano_$v.so ;; esac
  env $E PANO_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:---steps 10 --warmup 2} > "gpurun_out/abb_$v.txt" 2>&1 || exit $?
  python3 -c "
import json,sys;d=json.loads(open('gpurun_out/abb_$v.txt').read().strip().split('\n')[-1]);print('$v', d['ms_per_step'], json.dumps(d['kernels_ms_per_step']))"
done
