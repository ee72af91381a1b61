#!/bin/bash
# GPU-box: policy + rollout parity tests, then config-2 timing.  Each GPU step is time-limited;
# anything but a clean pass/fail stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest ${PYTEST_SEL:-tests/test_gpu_policy.py tests/test_gpu_rollout.py} \
  -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_policy.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_policy.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python tools/rollout_timing.py > gpurun_out/rollout_timing.log 2>&1
rc=$?; echo "timing rc=$rc"; cat gpurun_out/rollout_timing.log | grep -v amdgpu.ids
for lib in build_variants/libfenv_*.so; do
  [ -e "$lib" ] || continue
  FENV_LIB_OVERRIDE=$PWD/$lib timeout -k 10 200 python tools/rollout_timing.py > gpurun_out/rt_variant.log 2>&1
  rc=$?; echo "variant $lib rc=$rc"; grep -v amdgpu.ids gpurun_out/rt_variant.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
