#!/bin/bash
# tools/feat_time.py for the working build and each tools/ab variant in $VARIANTS
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in base ${VARIANTS}; do
  L=""; [ $v != base ] && L=tools/ab/libpano_$v.so
  PANO_LIB=$L timeout -k 10 120 python tools/feat_time.py ${WORK:-parrington} ${REPS:-10} 2>&1 | tail -1 || exit $?
done
