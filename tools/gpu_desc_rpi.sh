#!/bin/bash
# Descriptor fixed-point variant: parity tests on the default build, then class times A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_config5.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/t_rpi.txt 2>&1
echo "tests rc=$? $(tail -1 gpurun_out/t_rpi.txt)"
[ -s gpurun_out/t_rpi.txt ] && grep -E "FAIL|Error" gpurun_out/t_rpi.txt | head -5
for r in 1 2; do
for w in parrington synthetic; do
  for lib in vfx_image_stitching_amd/libpano.so tools/ab/libpano_rpi0.so; do
    echo "$w $(basename $lib) $(PANO_LIB=$lib timeout -k 10 200 python3 tools/feat_time.py $w 5 2>&1 | tail -1 | grep -o "'descriptor': [0-9.]*")"
  done
done
done
