#!/bin/bash
# JPEG decode knobs: subsequences per warm thread (PANO_JPEG_CHAIN) x warm-up window in MCUs (PANO_JPEG_WARM_MCUS).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for c in 1 2 3 4; do for w in 1 2 3 4; do
  echo "chain=$c warm=$w $(PANO_JPEG_CHAIN=$c PANO_JPEG_WARM_MCUS=$w timeout -k 10 100 python3 tools/jpeg_host_time.py 10 2>&1 | grep decode_call)"
done; done
