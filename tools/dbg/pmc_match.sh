cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcm
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $set --kernel-include-regex "dist_u8" --output-format csv -d gpurun_out/pmcm/p$i -o run -- python3 tools/dbg/prof_syn.py 1 > gpurun_out/pmcm/p$i.log 2>&1 || exit $?
done
python3 tools/pmc_summary.py gpurun_out/pmcm
