#!/bin/bash
# The fused PPO update's FIRST launch in a fresh process (bench.py's ppo_update line), sampled
# ROUNDS times for the library in $V and for the in-tree one, alternating
# (tools/ppo_first_update.py: wall time, outcome, re-runs).  A crash or a time limit stops it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=${V:-$PWD/build_variants/libfenv_prev.so}
run() {
  timeout -k 10 120 python tools/ppo_first_update.py "$1" > gpurun_out/first_update.log 2>&1
  rc=$?; tail -1 gpurun_out/first_update.log; [ $rc -eq 0 ]
}
for k in $(seq "${ROUNDS:-8}"); do
  FENV_LIB_OVERRIDE=$V run "$(basename "$V" .so)" || exit $?
  run in-tree || exit $?
done
