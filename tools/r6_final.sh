#!/bin/bash
# Round-6 evidence, in two GPU calls (each under gpurun's 20-minute limit):
#   PART=a  every -m gpu test, smoke(), PMC traffic per class and per launch (parrington and
#           synthetic 1080p), the default bench line (parrington)
#   PART=b  the synthetic 1080p bench line, the strong 144-frame N = 1 line, rocprofv3 kernel
#           stats of the parrington and 1080p benches, the one-step parrington timeline
# Everything lands in gpurun_out/final/; copy what is judged into profiles/ (r06_*).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/final; mkdir -p $O
if [ "${PART:-a}" = a ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -n 2 $O/pytest_gpu.txt
  [ $rc -ne 0 ] && exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -n 2 $O/smoke.txt
  [ $rc -ne 0 ] && exit $rc
  for w in parrington synthetic; do
    D=$O/pmc_$w; rm -rf $D; mkdir -p $D
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $D/$c -o run -- python3 tools/prof_features.py 3 $w > $D/$c.log 2>&1 || { echo "pmc $w $c failed"; exit 1; }
    done
    python3 tools/pmc_traffic.py $D 3 $w > $O/pmc_traffic_$w.json || exit 1
    python3 tools/pmc_per_launch.py $D 3 $w > $O/pmc_per_launch_$w.txt || exit 1
    tail -1 $O/pmc_per_launch_$w.txt
  done
  timeout -k 10 600 python bench.py > $O/bench_parrington.txt 2> $O/bench_parrington.err || { tail -5 $O/bench_parrington.err; exit 1; }
  tail -1 $O/bench_parrington.txt | cut -c1-300
else
  timeout -k 10 600 python bench.py --workload synthetic --steps 10 --warmup 2 > $O/bench_synthetic.txt 2> $O/bench_synthetic.err || { tail -5 $O/bench_synthetic.err; exit 1; }
  tail -1 $O/bench_synthetic.txt | cut -c1-300
  timeout -k 10 900 python bench.py --workload synthetic --scaling strong --steps 3 --warmup 1 > $O/bench_synthetic_strong.txt 2> $O/bench_synthetic_strong.err || { tail -5 $O/bench_synthetic_strong.err; exit 1; }
  tail -1 $O/bench_synthetic_strong.txt | cut -c1-300
  for w in parrington synthetic; do
    A="--steps 10 --warmup 2 --no-cpu-baseline"; [ $w = synthetic ] && A="--workload synthetic --steps 4 --warmup 1 --no-cpu-baseline"
    rm -rf $O/prof_$w
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$w -o run -- python3 bench.py $A > $O/prof_$w.log 2>&1 || { echo "prof $w failed"; exit 1; }
    python3 tools/kstats_step.py $O/prof_$w/run_kernel_stats.csv > $O/kernel_table_$w.txt
    head -3 $O/kernel_table_$w.txt
  done
  rm -rf $O/steps
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/steps -o run -- python3 tools/step_timeline.py > $O/steps.log 2>&1 || exit 1
  python3 tools/timeline.py $O/steps/run_kernel_trace.csv --step 10 > $O/timeline_parrington.txt
  tail -1 $O/timeline_parrington.txt
fi
echo "final part ${PART:-a} done"
