#!/bin/bash
# One GPU call for a kernel-variant decision: the in-tree library's GPU tests, then every
# build_variants/libfenv_*.so interleaved over ROUNDS rounds -- env rollouts at BASELINE configs
# 1/4/3 (tools/env_cfg_ab.py) and the fused policy rollout at config 2 (tools/pr_ab.py).
# PARITY_LIBS: variant libraries whose parity subset (PARITY_TESTS) runs first.  Any failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-variant}
mkdir -p "$O"
export PYTHONUNBUFFERED=1
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > "$O/pytest_gpu.log" 2>&1
  rc=$?; tail -2 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
fi
for lib in ${PARITY_LIBS:-}; do
  FENV_LIB_OVERRIDE=$PWD/$lib timeout -k 10 300 python -u -m pytest \
    ${PARITY_TESTS:-tests/test_gpu_parity.py tests/test_gpu_fullsize.py} -m gpu -q -x --timeout 200 \
    --timeout-method thread > "$O/parity_$(basename "$lib" .so).log" 2>&1
  rc=$?; echo "parity $lib rc=$rc"; tail -2 "$O/parity_$(basename "$lib" .so).log"
  [ $rc -le 1 ] || exit $rc  # a plain test failure is reported; crashes / timeouts stop here
done
for round in $(seq 1 ${ROUNDS:-3}); do
  for lib in build_variants/libfenv_*.so; do
    FENV_LIB_OVERRIDE=$PWD/$lib timeout -k 10 120 python tools/env_cfg_ab.py 2>/dev/null || exit $?
    [ "${POLICY:-1}" = 1 ] || continue
    FENV_LIB_OVERRIDE=$PWD/$lib timeout -k 10 120 python tools/pr_ab.py 2>/dev/null || exit $?
  done
done
