#!/bin/bash
# Descriptor register budget at 1080p: working tree (3 waves/SIMD) against 4, same box.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/desc1080
mkdir -p $O
for i in 1 2; do
  for lib in vfx_image_stitching_amd/libpano.so tools/ab/libpano_docc4.so; do
    tag=$(basename $lib .so)_$i
    PANO_LIB=$lib timeout -k 10 300 python3 bench.py --workload synthetic --steps 8 --warmup 2 --no-cpu-baseline > $O/bench_$tag.txt 2>&1
    rc=$?
    echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$tag.txt | head -1) $(grep -o '"descriptor": [0-9.]*' $O/bench_$tag.txt | head -1)"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
