#!/bin/bash
# The fused PPO update: the library in $V (default build_variants/libfenv_split0.so, the
# one-workgroup kernel, -DFENV_PPO_SPLIT=0) vs the in-tree one (split over two CUs): the PPO GPU
# tests on the variant, then PAIRS interleaved timing pairs of bench.py's ppo_update line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
V=${V:-$PWD/build_variants/libfenv_split0.so}
FENV_LIB_OVERRIDE=$V timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu \
  tests/test_gpu_rollout.py tests/test_gpu_training.py > gpurun_out/pt_ppo_split.log 2>&1
rc=$?; tail -3 gpurun_out/pt_ppo_split.log; [ $rc -le 1 ] || exit $rc
run() {
  timeout -k 10 120 python -c "import sys; sys.argv=['x']; import bench, torch, pkgload; \
pkg = pkgload.load(); r = bench.ppo_update_bench(pkg.__name__, torch.device('cuda', 0)); \
print('$1', round(r['us_per_minibatch'], 2), 'us/minibatch', round(r['ms_per_update'], 1), 'ms/update', flush=True)"
}
for k in $(seq "${PAIRS:-3}"); do
  FENV_LIB_OVERRIDE=$V run "$(basename "$V" .so)" || exit $?
  run in-tree || exit $?
done
