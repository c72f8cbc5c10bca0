#!/bin/bash
# JPEG file-to-file leg (tools/jpeg_host_time.py: decode call / decode GPU / stitch / encode)
# of the working tree against variants; SPECS may hold several settings joined by commas.
#   VARIANTS="env:PANO_JPEG_CHAIN=2,PANO_JPEG_WARM_MCUS=2 lib:sb256" bash tools/gpu_jpeg_ab.sh
# (round-4 uses: warm-up window x chain sweep, subsequence sizes, staging depth)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 300 python -u -m pytest $TESTS -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/tj_ab.txt 2>&1
  rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/tj_ab.txt)"; [ $rc -ne 0 ] && exit $rc
fi
for i in $(seq 1 ${REPS:-2}); do
  for v in base ${VARIANTS:-}; do
    case $v in
      base) spec="PANO_NONE=0"; lib=vfx_image_stitching_amd/libpano.so ;;
      lib:*) spec="PANO_NONE=0"; lib=tools/ab/libpano_${v#lib:}.so ;;
      env:*) spec=$(echo ${v#env:} | tr ',' ' '); lib=vfx_image_stitching_amd/libpano.so ;;
    esac
    out=$( (export $spec; PANO_LIB=$lib timeout -k 10 200 python3 tools/jpeg_host_time.py 20 2>&1) )
    rc=$?
    echo "$v rc=$rc $(echo "$out" | grep decode_call)"
    [ $rc -ne 0 ] && { echo "$out" | tail -5; exit $rc; }
  done
done
exit 0
