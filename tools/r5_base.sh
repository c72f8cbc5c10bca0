cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5base; rm -rf $O; mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.txt 2>&1 || exit $?
tail -1 $O/bench.txt | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/steps -o run -- python3 tools/step_timeline.py > $O/steps.log 2>&1 || exit $?
python3 tools/timeline.py $O/steps/run_kernel_trace.csv --step 10 > $O/timeline_parrington.txt
tail -3 $O/timeline_parrington.txt
