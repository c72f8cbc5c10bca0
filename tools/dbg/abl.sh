cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for v in base abl1 abl2; do
  if [ $v = base ]; then L=""; else L=tools/ab/libpano_$v.so; fi
  PANO_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abl_$v -o run -- python3 tools/prof_features.py 3 > gpurun_out/abl_$v.log 2>&1 || exit $?
  grep -h "descriptor\|orientation" gpurun_out/abl_$v/run_kernel_stats.csv | cut -d, -f1-5 | sed "s/^/$v /"
done
