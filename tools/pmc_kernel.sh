#!/bin/bash
# rocprofv3 SQ counter passes (counters only with --kernel-trace, one pass per set) over a
# short bench run, for the kernels matching $KRE; summaries in gpurun_out/pmck/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/pmck
rm -rf $O && mkdir -p $O
RE=${KRE:-blur_chain}
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --kernel-include-regex "$RE" --output-format csv -d $O/p$i -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --roofline-kernel blur_level --no-graph > $O/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
python3 tools/pmc_summary.py $O 2>&1 | tail -40
