#!/bin/bash
# Env-switch A/B of the parrington bench in one GPU call: each line of AB_TXT is a set of
# VAR=value assignments (or "base"); every variant runs ROUNDS times, interleaved.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/ab; rm -rf $O; mkdir -p $O
IFS=$'\n' read -r -d '' -a V <<< "${AB_TXT:-base}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in "${V[@]}"; do
    envs=(); [ "$v" != "base" ] && read -r -a envs <<< "$v"
    env "${envs[@]}" timeout -k 10 240 python bench.py --no-cpu-baseline --steps ${STEPS:-50} ${BENCH_ARGS:-} > $O/run.txt 2>&1 || { tail -5 $O/run.txt; exit 1; }
    ms=$(tail -1 $O/run.txt | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')
    echo "r$r [$v] ms_per_step=$ms" | tee -a $O/summary.txt
  done
done
