#!/bin/bash
# The fused PPO update's FIRST launch in a fresh process (bench.py's ppo_update line), sampled
# ROUNDS times for the library in $V and for the in-tree one, alternating.  A run that ends in
# a Python error (rc 1: NaN update) is counted and the sampling goes on; anything else (a
# crash, a time limit) stops it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=${V:-$PWD/build_variants/libfenv_prev.so}
run() {
  timeout -k 10 120 python -c "import sys; sys.argv=['x']; import bench, torch, pkgload; \
pkg = pkgload.load(); r = bench.ppo_update_bench(pkg.__name__, torch.device('cuda', 0), updates=1); \
print('$1', round(r['us_per_minibatch'], 2), 'us/minibatch', 'reruns', r.get('exchange_reruns'), flush=True)" \
    > gpurun_out/first_update.log 2>&1
  rc=$?
  if [ $rc -eq 0 ]; then tail -1 gpurun_out/first_update.log; else echo "$1 rc=$rc: $(tail -1 gpurun_out/first_update.log)"; fi
  [ $rc -le 1 ]
}
for k in $(seq "${ROUNDS:-8}"); do
  FENV_LIB_OVERRIDE=$V run "$(basename "$V" .so)" || exit $?
  run in-tree || exit $?
done
