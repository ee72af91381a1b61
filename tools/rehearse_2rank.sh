#!/bin/bash
# Rehearse bench.py's N > 1 path on a one-GPU box: two ranks on cuda:0 over gloo
# (FENV_DIST_BACKEND=gloo; RCCL refuses two ranks on one GPU).  Exercises the barrier, the
# max-over-ranks timing and the stats all-reduce; the rate says nothing about scaling.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2
FENV_DIST_BACKEND=gloo timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 \
  --formations 262144 > gpurun_out/r2/rehearse_2rank.json 2> gpurun_out/r2/rehearse_2rank.err
rc=$?; echo "2-rank rc=$rc"; cat gpurun_out/r2/rehearse_2rank.json | cut -c1-600; tail -3 gpurun_out/r2/rehearse_2rank.err
exit $rc
