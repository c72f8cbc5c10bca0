#!/bin/bash
# HBM traffic per kernel class for the SIFT step of $WORK (parrington | synthetic): two separate --pmc passes
# (FETCH_SIZE, WRITE_SIZE; kernel-trace only) over N stitches, corrected per
# profiles/r01_fetch_calibration.txt (bytes = 2 * FETCH_SIZE KB * 1024 + WRITE_SIZE KB * 1024),
# written to gpurun_out/pmc_traffic.json (bench.py reads a committed copy from profiles/).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
N=${N:-3}
W=${WORK:-parrington}
rm -rf gpurun_out/pmct && mkdir -p gpurun_out/pmct
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $c --output-format csv -d gpurun_out/pmct/$c -o run -- python3 tools/prof_features.py $N $W > gpurun_out/pmct/$c.log 2>&1 || exit $?
done
python3 tools/pmc_traffic.py gpurun_out/pmct $N $W > gpurun_out/pmc_traffic_$W.json && cat gpurun_out/pmc_traffic_$W.json
