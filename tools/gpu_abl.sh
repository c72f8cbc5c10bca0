#!/bin/bash
# Feature-stage class times (tools/feat_time.py, no matching) of the working tree and each
# tools/ab/libpano_*.so variant, on parrington and synthetic 1080p.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for w in ${WORKLOADS:-parrington synthetic}; do for v in vfx_image_stitching_amd/libpano.so tools/ab/libpano_*.so; do
  echo "$w $(basename $v) $(PANO_LIB=$v timeout -k 10 200 python3 tools/feat_time.py $w 5 2>&1 | tail -1 | grep -o "'blur_level'.*")"
done; done
