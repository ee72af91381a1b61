#!/bin/bash
# Config-1/3/4 env rollout A/B: parity of the variant builds, then build_variants/libfenv_*.so
# interleaved (tools/env_cfg_ab.py), ROUNDS rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for lib in ${PARITY_LIBS:-}; do
  FENV_LIB_OVERRIDE=$PWD/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py \
    tests/test_gpu_fullsize.py -m gpu -q -x --timeout 200 --timeout-method thread \
    -k "golden or extreme or full_size or config1 or rollout_chunks" 2>&1 | tail -2
  [ ${PIPESTATUS[0]} -eq 0 ] || exit 1
done
for round in $(seq 1 ${ROUNDS:-3}); do
  for lib in build_variants/libfenv_*.so; do
    FENV_LIB_OVERRIDE=$PWD/$lib timeout -k 10 120 python tools/env_cfg_ab.py 2>/dev/null || exit $?
  done
done
