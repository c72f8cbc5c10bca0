#!/bin/bash
# JPEG file-to-file leg under decode knobs (tools/jpeg_host_time.py), one process per setting.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for spec in "PANO_NONE=0" ${SPECS:-"PANO_JPEG_WARM_MCUS=3" "PANO_JPEG_WARM_MCUS=2" "PANO_JPEG_WARM_MCUS=6" "PANO_JPEG_CHAIN=2"}; do
  echo "$spec $( (export $spec; timeout -k 10 200 python3 tools/jpeg_host_time.py 20 2>&1 | grep decode_call) )"
done
