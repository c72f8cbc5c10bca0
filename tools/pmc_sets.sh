#!/bin/bash
# rocprofv3 counter passes (one pass per set, counters only with --kernel-trace) over a short
# eager bench run, for the kernels matching $KRE; summaries in gpurun_out/$OUT/.
#   KRE=dist_i8 BENCH_ARGS="--workload synthetic" SETS="SQ_WAVES SQ_INSTS_VALU;SQ_BUSY_CYCLES" bash tools/pmc_sets.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-pmcs}
rm -rf $O && mkdir -p $O
IFS=';' read -ra SETV <<< "${SETS:?counter sets}"
i=0
for set in "${SETV[@]}"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $set --kernel-include-regex "${KRE:?kernel regex}" --output-format csv -d $O/p$i -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-graph ${BENCH_ARGS:-} > $O/p$i.log 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc"
  [ $rc -ne 0 ] && { tail -3 $O/p$i.log; exit $rc; }
done
python3 tools/pmc_summary.py $O > $O/summary.txt 2>&1
head -60 $O/summary.txt
