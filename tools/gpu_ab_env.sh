#!/bin/bash
# A/B of two environment settings on the same box: rocprofv3 kernel stats of bench.py under
# each, then the per-step kernel tables side by side.
#   A="PANO_BLUR_CASCADE=0" B="PANO_BLUR_CASCADE=1" BENCH_ARGS="" bash tools/gpu_ab_env.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for tag in A B; do
  spec=${!tag}
  rm -rf gpurun_out/ab_$tag
  ( export $spec; timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_$tag -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_$tag.log 2>&1 )
  rc=$?; echo "$tag ($spec) rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$tag.log | head -1)"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/ab_$tag.log; exit $rc; }
  python3 tools/kstats_step.py gpurun_out/ab_$tag/run_kernel_stats.csv plan_device 4 > gpurun_out/ab_$tag.txt
  head -${TOP:-14} gpurun_out/ab_$tag.txt
done
