#!/bin/bash
# One GPU call: the whole -m gpu suite, then alternating bench lines of the working tree against
# variants (a library built with other flags, or an environment setting), per workload.
#   VARIANTS="lib:nostag env:PANO_DESC_OCC=3" WORKLOADS="parrington synthetic" bash tools/gpu_r4a.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r4a
mkdir -p $O
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -n 4 $O/pytest.txt
  [ $rc -ne 0 ] && exit $rc
fi
for wl in ${WORKLOADS:-parrington synthetic}; do
  for i in 1 2; do
    for v in base ${VARIANTS:-}; do
      case $v in
        base) spec="PANO_NONE=0"; lib=vfx_image_stitching_amd/libpano.so ;;
        lib:*) spec="PANO_NONE=0"; lib=tools/ab/libpano_${v#lib:}.so ;;
        env:*) spec=${v#env:}; lib=vfx_image_stitching_amd/libpano.so ;;
      esac
      tag=${wl}_$(echo $v | tr ':=' '__')_$i
      ( export $spec; PANO_LIB=$lib timeout -k 10 300 python3 bench.py --workload $wl --steps ${STEPS:-40} --warmup 3 --no-cpu-baseline > $O/bench_$tag.txt 2>&1 )
      rc=$?
      echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$tag.txt | head -1) $(grep -o '"kernels_ms_per_step": {[^}]*}' $O/bench_$tag.txt | head -1)"
      [ $rc -ne 0 ] && { tail -5 $O/bench_$tag.txt; exit $rc; }
    done
  done
done
exit 0
