#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration passes (separate --pmc runs, kernel-trace only).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/calib
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/calib/f -o run -- ./tools/calib/fetch_calib > gpurun_out/calib/f.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/calib/w -o run -- ./tools/calib/fetch_calib > gpurun_out/calib/w.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob
for d in ("f", "w"):
    for f in glob.glob(f"gpurun_out/calib/{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            print(d, r["Kernel_Name"].split("(")[0], r["Counter_Name"], float(r["Counter_Value"]) * 1024 / (512 << 20))
PY
