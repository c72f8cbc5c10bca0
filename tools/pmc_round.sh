#!/bin/bash
# rocprofv3 PMC passes (counters only with --kernel-trace; no sys/runtime trace).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
RE=${KRE:-extrema_scan|localize|descriptor|orientation|blur_level|dist_mfma}
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_FLAT GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" ${EXTRA_SETS:-}; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --kernel-include-regex "$RE" --output-format csv -d gpurun_out/pmc/p$i -o run -- python3 tools/prof_features.py 3 > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done
