#!/bin/bash
# Tail check: GPU parity subset, per-level stamps of blur_tail (solo / beside the extrema
# scan), then bench A/B of the working tree against tools/ab/libpano_HEAD.so.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/tail
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stages.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 $O/pytest.txt
[ $rc -ne 0 ] && exit $rc
for solo in 1 0; do
  if [ $solo = 1 ]; then export PANO_TAIL_SOLO=1; else unset PANO_TAIL_SOLO; fi
  PANO_LIB=tools/ab/libpano_tailclk.so timeout -k 10 180 python3 -u tools/tail_clock.py > $O/clk_solo$solo.txt 2>&1
  rc=$?; echo "solo=$solo rc=$rc"; tail -n 2 $O/clk_solo$solo.txt
  [ $rc -ne 0 ] && exit $rc
done
unset PANO_TAIL_SOLO
for i in 1 2; do
  for lib in vfx_image_stitching_amd/libpano.so tools/ab/libpano_HEAD.so; do
    tag=$(basename $lib .so)_$i
    PANO_LIB=$lib timeout -k 10 240 python3 bench.py --steps 40 --warmup 3 --no-cpu-baseline > $O/bench_$tag.txt 2>&1
    rc=$?
    echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$tag.txt | head -1) $(grep -o '"blur_level": [0-9.]*' $O/bench_$tag.txt | head -1) $(grep -o '"extrema_localize": [0-9.]*' $O/bench_$tag.txt | head -1)"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
