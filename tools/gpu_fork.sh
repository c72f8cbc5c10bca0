#!/bin/bash
# PANO_OCT_FORK: parity subset with the fork on, then bench lines for fork settings.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/fork
mkdir -p $O
PANO_OCT_FORK=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread -k "pyramid or end_to_end or graph_replay or determinism or sift" > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 $O/pytest.txt
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for fk in -1 0 1 2; do
    PANO_OCT_FORK=$fk timeout -k 10 240 python3 bench.py --steps 40 --warmup 3 --no-cpu-baseline > $O/bench_${fk}_$i.txt 2>&1
    rc=$?
    echo "fork=$fk/$i rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${fk}_$i.txt | head -1) $(grep -o '"blur_level": [0-9.]*' $O/bench_${fk}_$i.txt | head -1)"
    [ $rc -ne 0 ] && exit $rc
  done
done

for i in 1 2; do
  for lib in vfx_image_stitching_amd/libpano.so tools/ab/libpano_docc5.so tools/ab/libpano_docc3.so; do
    tag=$(basename $lib .so)_$i
    PANO_LIB=$lib timeout -k 10 240 python3 bench.py --steps 40 --warmup 3 --no-cpu-baseline > $O/bench_$tag.txt 2>&1
    rc=$?
    echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$tag.txt | head -1) $(grep -o '"descriptor": [0-9.]*' $O/bench_$tag.txt | head -1)"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
