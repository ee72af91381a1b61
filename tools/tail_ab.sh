#!/bin/bash
# Fused policy rollout: parity of the FENV_PR_TAIL=1 build, then same-box timing of
# build_variants/libfenv_pol_*.so interleaved (tools/rollout_timing.py, config 2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
FENV_LIB_OVERRIDE=$PWD/build_variants/libfenv_pol_tail.so timeout -k 10 300 python -u -m pytest \
  tests/test_gpu_rollout.py tests/test_gpu_fullsize.py -k "fused or policy_rollout or collect" \
  -x -q --timeout 150 --timeout-method thread || exit $?
for round in $(seq 1 ${ROUNDS:-3}); do
  for lib in build_variants/libfenv_pol_*.so; do
    echo "$lib:"; FENV_LIB_OVERRIDE=$PWD/$lib timeout -k 10 90 python tools/rollout_timing.py 2>/dev/null | grep fused=True || exit $?
  done
done
