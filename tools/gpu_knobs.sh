#!/bin/bash
# Environment-knob sweep on one box (bench lines, parrington): each setting twice, interleaved.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/knobs
mkdir -p $O
SETS=("X=0" "PANO_EXTREMA_STREAM_MIN_H=96" "PANO_EXTREMA_STREAM_MIN_H=48" "PANO_BLUR_SMALL=1000" "PANO_EXTREMA_XSR=16")
for i in 1 2; do
  for s in "${SETS[@]}"; do
    tag=$(echo $s | tr '=' '_')_$i
    env $s timeout -k 10 240 python3 bench.py --steps 40 --warmup 3 --no-cpu-baseline > $O/bench_$tag.txt 2>&1
    rc=$?
    echo "$s/$i rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$tag.txt | head -1) $(grep -o '"blur_level": [0-9.]*' $O/bench_$tag.txt | head -1) $(grep -o '"extrema_localize": [0-9.]*' $O/bench_$tag.txt | head -1)"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
