#!/bin/bash
# Parity (policy + fused rollout GPU tests) of one library variant, then the interleaved
# config-2 timing of every build_variants/libfenv_pol_*.so (tools/policy_persist_ab.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2
for lib in ${PARITY_LIBS:-}; do
  FENV_LIB_OVERRIDE=$PWD/$lib timeout -k 10 400 python -u -m pytest tests/test_gpu_policy.py \
    tests/test_gpu_rollout.py tests/test_gpu_fullsize.py -m gpu -q -x --timeout 200 \
    --timeout-method thread -k "not two_rank and not beyond_int32" 2>&1 | tail -3
  [ ${PIPESTATUS[0]} -eq 0 ] || exit 1
done
ROUNDS=${ROUNDS:-3} bash tools/policy_persist_ab.sh
