#!/bin/bash
# One GPU call refreshing the committed measurements: bench lines (parrington, synthetic 1080p),
# rocprofv3 kernel stats of both, the one-step timeline, PMC HBM traffic per class (parrington).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/refresh
rm -rf $O && mkdir -p $O
timeout -k 10 600 python bench.py > $O/bench_parrington.txt 2>&1 || exit $?
tail -1 $O/bench_parrington.txt
timeout -k 10 600 python bench.py --workload synthetic --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_synthetic.txt 2>&1 || exit $?
tail -1 $O/bench_synthetic.txt | cut -c1-300
for w in parrington synthetic; do
  A="--steps 10 --warmup 2 --no-cpu-baseline"; [ $w = synthetic ] && A="--workload synthetic --steps 4 --warmup 1 --no-cpu-baseline"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$w -o run -- python3 bench.py $A > $O/prof_$w.log 2>&1 || exit $?
done
K=$(find $O/prof_parrington -name "*kernel_trace.csv" | head -1)
python3 tools/timeline.py $K --step 6 > $O/timeline_parrington.txt
bash tools/pmc_traffic.sh > $O/pmc_traffic.log 2>&1 || exit $?
cp gpurun_out/pmc_traffic.json $O/
echo refresh done
