#!/bin/bash
# GPU-box: policy + rollout parity tests (skip with SKIP_TESTS=1), then config-2 timing of the
# in-tree library and of every build_variants/libfenv_*.so.  Each GPU step is time-limited;
# anything but a clean pass/fail stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest ${PYTEST_SEL:-tests/test_gpu_policy.py tests/test_gpu_rollout.py} \
    -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_policy.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_policy.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
for F in ${TIMING_F:-65536}; do
  timeout -k 10 200 python tools/rollout_timing.py $F > gpurun_out/rollout_timing.log 2>&1
  rc=$?; echo "timing F=$F rc=$rc"; grep -v amdgpu.ids gpurun_out/rollout_timing.log
  if [ $rc -ne 0 ]; then exit $rc; fi
  for lib in build_variants/libfenv_*.so; do
    [ -e "$lib" ] || continue
    FENV_LIB_OVERRIDE=$PWD/$lib timeout -k 10 200 python tools/rollout_timing.py $F > gpurun_out/rt_variant.log 2>&1
    rc=$?; echo "variant $lib F=$F rc=$rc"; grep "fused=True\|policy_forward" gpurun_out/rt_variant.log
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
