#!/bin/bash
# A/B on one box: GPU parity subset on the working tree, then alternating bench runs of the
# working tree's libpano.so and tools/ab/libpano_$AB.so (per-class kernel times included).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/ab
mkdir -p $O
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_stages.py} -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -n 3 $O/pytest.txt
  [ $rc -ne 0 ] && exit $rc
fi
for i in 1 2; do
  for lib in vfx_image_stitching_amd/libpano.so tools/ab/libpano_$AB.so; do
    tag=$(basename $lib .so)_$i
    PANO_LIB=$lib timeout -k 10 240 python3 bench.py --steps 40 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > $O/bench_$tag.txt 2>&1
    rc=$?
    echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$tag.txt | head -1) $(grep -o '"kernels_ms_per_step": {[^}]*}' $O/bench_$tag.txt | head -1)"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
