#!/bin/bash
# Cascade vs level-by-level kernel tables (rocprof) at parrington and 1080p, then the
# strong-scaling N=1 bench line (144-frame synthetic batch, with cpu_baseline).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r4b
mkdir -p $O
for wl in parrington synthetic; do
  A="PANO_BLUR_CASCADE=0" B="PANO_BLUR_CASCADE=1" BENCH_ARGS="--workload $wl" TOP=40 bash tools/gpu_ab_env.sh > $O/cas_$wl.txt 2>&1
  rc=$?; grep "rc=" $O/cas_$wl.txt
  [ $rc -ne 0 ] && exit $rc
  cp gpurun_out/ab_A.txt $O/cas_${wl}_off.txt; cp gpurun_out/ab_B.txt $O/cas_${wl}_on.txt
done
timeout -k 10 600 python3 bench.py --workload synthetic --scaling strong --steps 3 --warmup 1 > $O/strong.txt 2>&1
rc=$?; echo "strong rc=$rc"; tail -c 1500 $O/strong.txt
exit $rc
