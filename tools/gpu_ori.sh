#!/bin/bash
# Orientation prefetch A/B: parity subset on the working tree, then bench lines of the working
# tree (prefetch, 4 workgroups/CU budget), the 5-workgroup budget and the old form.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/ori
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread -k "sift or end_to_end or graph or determinism" > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 $O/pytest.txt
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for lib in vfx_image_stitching_amd/libpano.so tools/ab/libpano_ori5.so tools/ab/libpano_orioff.so; do
    tag=$(basename $lib .so)_$i
    PANO_LIB=$lib timeout -k 10 240 python3 bench.py --steps 40 --warmup 3 --no-cpu-baseline > $O/bench_$tag.txt 2>&1
    rc=$?
    echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$tag.txt | head -1) $(grep -o '"orientation": [0-9.]*' $O/bench_$tag.txt | head -1)"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
