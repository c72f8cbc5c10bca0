#!/bin/bash
# Cache counters of the descriptor kernel, emit order vs locality order (PANO_DESC_ORDER):
# one rocprofv3 pass per counter set (TCP = L1, TCC = L2), counters only with --kernel-trace.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/pmcd
rm -rf $O && mkdir -p $O
for ord in 0 1; do
  i=0
  for set in "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_BUSY_CYCLES"; do
    i=$((i+1))
    PANO_DESC_ORDER=$ord timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --kernel-include-regex "descriptor_wave" --output-format csv -d $O/o${ord}/p$i -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --roofline-kernel descriptor --no-graph > $O/o${ord}_p$i.log 2>&1
    rc=$?; echo "order $ord pass $i rc=$rc"
    [ $rc -ne 0 ] && exit $rc
  done
  python3 tools/pmc_summary.py $O/o${ord} > $O/summary_order$ord.txt 2>&1; cat $O/summary_order$ord.txt | head -20
done
