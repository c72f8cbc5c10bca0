#!/bin/bash
# L1/L2 counters of kernels matching $KRE (one pass) for tools/prof_features.py.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/pmcc_${TAG:-base}; rm -rf $out; mkdir -p $out
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "${KRE:-descriptor}" --output-format csv -d $out/p1 -o run -- python3 tools/prof_features.py 2 > $out/p1.log 2>&1 || exit $?
python3 tools/pmc_summary.py $out
