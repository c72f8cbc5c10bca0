#!/bin/bash
# Round-6 GPU call: STAGES (space-separated, in order) of
#   tests  -- every -m gpu test (or TESTS=...)
#   pmc    -- FETCH_SIZE / WRITE_SIZE passes over N stitches of parrington and synthetic 1080p:
#             per-class traffic (tools/pmc_traffic.py) and the per-launch table of the pyramid
#             and extrema launches (tools/pmc_per_launch.py), into gpurun_out/r6/
#   ab     -- bench ms_per_step of the working tree against variant libraries (VARIANTS: names
#             of tools/ab/libpano_<name>.so), ROUNDS interleaved rounds, BENCH_ARGS
#   bench  -- the default bench line (BENCH_ARGS)
#   prof   -- rocprofv3 --kernel-trace --stats of bench (BENCH_ARGS) -> kernel table
# Every GPU step has its own time limit; the first failure ends the call.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6; mkdir -p $O
for st in ${STAGES:-tests}; do
  case $st in
  tests)
    timeout -k 10 ${TLIM:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1
    rc=$?; echo "pytest rc=$rc"; tail -n 3 $O/pytest.txt
    [ $rc -ne 0 ] && exit $rc ;;
  t2)   # a second test selection (TESTS2) whose failure is reported but does not end the call
    timeout -k 10 ${TLIM2:-300} python -u -m pytest ${TESTS2} -m gpu -x -v --timeout ${TTO2:-100} --timeout-method thread > $O/pytest2.txt 2>&1
    echo "pytest2 rc=$?"; tail -n 40 $O/pytest2.txt | cut -c1-300 ;;
  pmc)
    for w in ${WORKS:-parrington synthetic}; do
      D=$O/pmc_$w; rm -rf $D; mkdir -p $D
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $D/$c -o run -- python3 tools/prof_features.py ${N:-3} $w > $D/$c.log 2>&1 || { echo "pmc $w $c failed"; tail -5 $D/$c.log; exit 1; }
      done
      python3 tools/pmc_traffic.py $D ${N:-3} $w > $O/pmc_traffic_$w.json || exit 1
      python3 tools/pmc_per_launch.py $D ${N:-3} $w > $O/pmc_per_launch_$w.txt || exit 1
      tail -2 $O/pmc_per_launch_$w.txt
    done ;;
  ab)
    : > $O/ab_summary.txt
    for r in $(seq 1 ${ROUNDS:-2}); do
      for v in base ${VARIANTS:-}; do
        lib=""
        case $v in base) ;; env:*) lib="${v#env:}" ;; *) lib="PANO_LIB=tools/ab/libpano_$v.so" ;; esac
        env $lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-60} ${BENCH_ARGS:-} > $O/ab_run.txt 2> $O/ab_run.err || { tail -5 $O/ab_run.err; exit 1; }
        ms=$(tail -1 $O/ab_run.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d.get("kernels_ms_per_step", {}); print(d["ms_per_step"], d.get("single_context_ms_per_step"), "blur", k.get("blur_level"), "extrema", k.get("extrema_localize"), "desc", k.get("descriptor"))')
        echo "r$r [$v] ms_per_step single_context: $ms" | tee -a $O/ab_summary.txt
      done
    done ;;
  rehearse)   # the N > 1 bench path on this one-GPU box: N ranks on cuda:0 over gloo, no launcher
    PANO_BENCH_REHEARSE=1 timeout -k 10 ${TLIM_R:-900} python bench.py --gpus ${NR:-2} --steps 3 --warmup 1 > $O/rehearse_n${NR:-2}.txt 2> $O/rehearse_n${NR:-2}.err
    rc=$?; echo "rehearse rc=$rc"; tail -n 1 $O/rehearse_n${NR:-2}.txt | cut -c1-600; tail -n 3 $O/rehearse_n${NR:-2}.err
    [ $rc -ne 0 ] && exit $rc ;;
  bench)
    timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $O/bench.txt 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
    tail -1 $O/bench.txt | cut -c1-400 ;;
  prof)
    rm -rf $O/prof
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS:---steps 20 --warmup 2} > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
    python3 tools/kstats_step.py $(ls $O/prof/*kernel_stats.csv | head -1) > $O/kernel_table.txt 2>&1; head -25 $O/kernel_table.txt ;;
  *) echo "unknown stage $st"; exit 2 ;;
  esac
done
echo "r6_run done"
