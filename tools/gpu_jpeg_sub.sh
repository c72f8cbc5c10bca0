cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in vfx_image_stitching_amd/libpano.so tools/ab/libpano_sb256.so tools/ab/libpano_sb1024.so; do
  PANO_LIB=$v timeout -k 10 300 python -u -m pytest tests/test_jpeg.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/tj_$(basename $v).txt 2>&1
  echo "$(basename $v) tests rc=$? $(tail -1 gpurun_out/tj_$(basename $v).txt)"
  echo "$(basename $v) $(PANO_LIB=$v timeout -k 10 200 python3 tools/jpeg_host_time.py 20 2>&1 | grep decode_call)"
done
