#!/bin/bash
# Feature-stage class times (tools/feat_time.py: the SIFT feature chain without matching) of the
# working tree against variants, per workload; KEY picks the class printed.
#   VARIANTS="lib:rpi0 env:PANO_DESC_OCC=3" KEY=descriptor WORKLOADS="parrington synthetic" bash tools/gpu_feat_ab.sh
# (round-4 uses: descriptor budgets and fixed point, blur ablations with KEY=blur_level)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for i in $(seq 1 ${REPS:-2}); do
  for wl in ${WORKLOADS:-parrington synthetic}; do
    for v in base ${VARIANTS:-}; do
      case $v in
        base) spec="PANO_NONE=0"; lib=vfx_image_stitching_amd/libpano.so ;;
        lib:*) spec="PANO_NONE=0"; lib=tools/ab/libpano_${v#lib:}.so ;;
        env:*) spec=${v#env:}; lib=vfx_image_stitching_amd/libpano.so ;;
      esac
      out=$( (export $spec; PANO_LIB=$lib timeout -k 10 200 python3 tools/feat_time.py $wl 5 2>&1) )
      rc=$?
      echo "$wl $v rc=$rc $(echo "$out" | tail -1 | grep -o "'${KEY:-descriptor}': [0-9.]*")"
      [ $rc -ne 0 ] && { echo "$out" | tail -5; exit $rc; }
    done
  done
done
exit 0
