#!/bin/bash
# blur_octs timing ablations (PANO_OCTS_ABL bits: 1 no waits, 2 plain loads, 4 no store drain,
# 8 plain G stores; planes WRONG under any bit -- timing only) and workgroups per CU
# (PANO_OCTS_WGS), first octave (PANO_BLUR_OCTS): one kernel trace of graph-replayed parrington steps per variant.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
# VARIANTS: "abl wgs from" triples, one per line
IFS=$'\n' read -r -d '' -a VARIANTS <<< "${VARIANTS_TXT:-0 8 1}"
export TMPDIR=/tmp
O=gpurun_out/octs_abl; rm -rf $O; mkdir -p $O
for v in "${VARIANTS[@]:-0 8 1}"; do
  set -- $v
  tag=abl$1_wgs$2_from$3
  PANO_BLUR_OCTS=$3 PANO_OCTS_ABL=$1 PANO_OCTS_WGS=$2 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/$tag -o run -- python3 tools/step_timeline.py > $O/$tag.log 2>&1 || exit $?
  python3 tools/timeline.py $O/$tag/run_kernel_trace.csv --step 10 > $O/$tag.txt
  echo "$tag octs=$(grep -E 'blur_octs' $O/$tag.txt | awk '{print $2}') blur_sum=$(grep -E 'blur_(fast|octs)' $O/$tag.txt | awk '{s+=$2} END {print s}') $(tail -1 $O/$tag.txt | cut -c1-40)"
  rm -rf $O/$tag
done
