cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for v in ring2 ring2c1 ring3c1 ring4c1; do
  PANO_LIB=tools/ab/libpano_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "descriptor or feature or sift_pair or golden" > gpurun_out/ring_$v.txt 2>&1
  rc=$?; echo "$v pytest rc=$rc $(tail -1 gpurun_out/ring_$v.txt)"
  [ $rc -ne 0 ] && exit $rc
done
REPS=1 VARIANTS="lib:ring2 lib:ring2c1 lib:ring3c1 lib:ring4c1" KEY=descriptor bash tools/gpu_feat_ab.sh
