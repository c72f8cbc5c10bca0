#!/bin/bash
# Tail check: pyramid/SIFT parity subset, per-level stamps of blur_tail, bench lines of the
# side-stream octave split.
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
for so in 0 1 2 0 1 2; do
  PANO_SIDE_OCT=$so timeout -k 10 180 python3 bench.py --steps 40 --warmup 3 --no-cpu-baseline > $O/bench_side$so.txt 2>&1
  rc=$?; echo "side=$so rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/bench_side$so.txt | head -1) $(grep -o '"kernel_ms_per_step": [0-9.]*' $O/bench_side$so.txt | head -1)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
