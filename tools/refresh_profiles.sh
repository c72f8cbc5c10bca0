#!/bin/bash
# One GPU call refreshing the committed measurements of round $R (default r03):
#   PMC HBM traffic per kernel class (parrington and synthetic 1080p; copied into profiles/
#   first, so the bench lines below report it as roofline.traffic), the bench lines
#   (parrington; synthetic 1080p weak; synthetic strong N=1), rocprofv3 kernel stats of both
#   workloads, and the one-step timeline of parrington.  Everything lands in
#   gpurun_out/refresh/; copy what is judged into profiles/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${R:-r05}
O=gpurun_out/refresh
rm -rf $O && mkdir -p $O
for w in parrington synthetic; do
  WORK=$w N=3 bash tools/pmc_traffic.sh > $O/pmc_traffic_$w.log 2>&1 || { cat $O/pmc_traffic_$w.log | tail -5; exit 1; }
  cp gpurun_out/pmc_traffic_$w.json $O/${R}_pmc_traffic_$w.json
  cp gpurun_out/pmc_traffic_$w.json profiles/${R}_pmc_traffic_$w.json
done
echo "pmc done"
timeout -k 10 600 python bench.py > $O/bench_parrington.txt 2>&1 || exit $?
tail -1 $O/bench_parrington.txt | cut -c1-300
timeout -k 10 600 python bench.py --workload synthetic --steps 10 --warmup 2 > $O/bench_synthetic.txt 2>&1 || exit $?
tail -1 $O/bench_synthetic.txt | cut -c1-300
timeout -k 10 900 python bench.py --workload synthetic --scaling strong --steps 3 --warmup 1 > $O/bench_synthetic_strong.txt 2>&1 || exit $?
tail -1 $O/bench_synthetic_strong.txt | cut -c1-300
for w in parrington synthetic; do
  A="--steps 10 --warmup 2 --no-cpu-baseline"; [ $w = synthetic ] && A="--workload synthetic --steps 4 --warmup 1 --no-cpu-baseline"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$w -o run -- python3 bench.py $A > $O/prof_$w.log 2>&1 || exit $?
done
# the timeline of one graph-replayed step (only replays in that process)
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/steps -o run -- python3 tools/step_timeline.py > $O/steps.log 2>&1 || exit $?
python3 tools/timeline.py $O/steps/run_kernel_trace.csv --step 10 > $O/timeline_parrington.txt
tail -1 $O/timeline_parrington.txt
echo refresh done
