#!/bin/bash
# PMC passes (kernel regex $KRE) of tools/prof_features.py under the environment $ENVSET
# (VAR=value[,VAR=value]); output under gpurun_out/pmce_<tag>.  One counter set per pass.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
tag=$(echo "${ENVSET:-base}" | tr ',=' '__')
[ "${ENVSET:-base}" != base ] && for kv in ${ENVSET//,/ }; do export "$kv"; done
out=gpurun_out/pmce_$tag; rm -rf $out; mkdir -p $out
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --kernel-include-regex "${KRE:-blur}" --output-format csv -d $out/p$i -o run -- python3 tools/prof_features.py 2 > $out/p$i.log 2>&1 || exit $?
done
python3 tools/pmc_summary.py $out
