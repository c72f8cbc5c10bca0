#!/bin/bash
# Final evidence (tools/gpu_final.sh), then the cylindrical 4-rows-per-thread variant
# (tools/ab/libpano_cyl.so): its cylindrical / end-to-end GPU tests and a bench A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
bash tools/gpu_final.sh || exit $?
O=gpurun_out/cyl
mkdir -p $O
PANO_LIB=tools/ab/libpano_cyl.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread -k "cylindrical or end_to_end or bands or determinism" > $O/pytest.txt 2>&1
rc=$?; echo "cyl pytest rc=$rc"; tail -n 2 $O/pytest.txt
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for lib in vfx_image_stitching_amd/libpano.so tools/ab/libpano_cyl.so; do
    tag=$(basename $lib .so)_$i
    PANO_LIB=$lib timeout -k 10 240 python3 bench.py --steps 40 --warmup 3 --no-cpu-baseline > $O/bench_$tag.txt 2>&1
    rc=$?
    echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$tag.txt | head -1) $(grep -o '"cyl_gather": [0-9.]*' $O/bench_$tag.txt | head -1)"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
