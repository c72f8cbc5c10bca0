#!/bin/bash
# Descriptor class time (tools/feat_time.py) for library x PANO_DESC_OCC combinations.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for w in parrington synthetic; do
  for lib in vfx_image_stitching_amd/libpano.so tools/ab/libpano_*.so; do
    for occ in ${OCCS:-3 4}; do
      echo "$w $(basename $lib) occ=$occ $(PANO_DESC_OCC=$occ PANO_LIB=$lib timeout -k 10 200 python3 tools/feat_time.py $w 5 2>&1 | tail -1 | grep -o "'descriptor': [0-9.]*")"
    done
  done
done
