#!/bin/bash
# rocprofv3 counter passes over the feature stage alone (tools/feat_time.py: runs timing-ablation
# builds whose descriptors are garbage) per library variant; summaries in gpurun_out/$OUT/<v>/.
#   VARIANTS="rows0 dabl5" KRE=descriptor_wave SETS="TCP_TCC_READ_REQ_sum;TCC_HIT_sum TCC_MISS_sum" bash tools/pmc_feat.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
IFS=';' read -ra SETV <<< "${SETS:?counter sets}"
for v in ${VARIANTS:?variants}; do
  lib=tools/ab/libpano_$v.so; [ "$v" = base ] && lib=vfx_image_stitching_amd/libpano.so
  O=gpurun_out/${OUT:-pmcf}/$v
  rm -rf $O && mkdir -p $O
  i=0
  for set in "${SETV[@]}"; do
    i=$((i+1))
    PANO_LIB=$lib timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $set --kernel-include-regex "${KRE:?kernel regex}" --output-format csv -d $O/p$i -o run -- python3 tools/feat_time.py ${WORK:-parrington} 2 > $O/p$i.log 2>&1
    rc=$?; echo "$v pass $i ($set) rc=$rc"
    [ $rc -ne 0 ] && { tail -3 $O/p$i.log; exit $rc; }
  done
  python3 tools/pmc_summary.py $O > $O/summary.txt 2>&1
  echo "== $v"; head -40 $O/summary.txt
done
