#!/bin/bash
# The N > 1 bench path rehearsed on a one-GPU box: N ranks on cuda:0 over gloo
# (PANO_BENCH_REHEARSE=1): strong config 5 sharded over the ranks + the weak parrington laps.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
N=${N:-2}
PANO_BENCH_REHEARSE=1 timeout -k 10 ${TLIM:-600} python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
  --master-addr 127.0.0.1 --master-port ${PORT:-29571} bench.py --gpus $N --steps ${STEPS:-3} --warmup 1 \
  > gpurun_out/rehearse_n$N.txt 2>&1
rc=$?; echo "rehearse rc=$rc"; tail -n 2 gpurun_out/rehearse_n$N.txt | cut -c1-600
exit $rc
