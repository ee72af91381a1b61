#!/bin/bash
# Same-box A/B of the fused PPO update: the in-tree libfenv.so vs build_variants/libfenv_old.so
# (FENV_LIB_OVERRIDE), interleaved, PAIRS pairs; prints bench.py's ppo_update line per run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PAIRS=${PAIRS:-3}
run() {
  timeout -k 10 120 python -c "import sys; sys.argv=['x']; import bench, torch, pkgload; \
pkg = pkgload.load(); print('$1', bench.ppo_update_bench(pkg.__name__, torch.device('cuda', 0)), flush=True)"
}
for k in $(seq "$PAIRS"); do
  run new || exit $?
  FENV_LIB_OVERRIDE=$PWD/build_variants/libfenv_old.so run old || exit $?
done
