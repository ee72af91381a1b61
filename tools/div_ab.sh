#!/bin/bash
# Same-box A/B for a library change: env rollout (tools/env_ab.sh, in-tree vs build_variants/
# libfenv_*.so) and the config-2 fused policy rollout (tools/rollout_timing.py) with the in-tree
# library and each build_variants/libfenv_pol_*.so, interleaved over ROUNDS rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROUNDS=${ROUNDS:-3} bash tools/env_ab.sh || exit $?
for round in $(seq 1 ${ROUNDS:-3}); do
  echo "policy in-tree:"; timeout -k 10 90 python tools/rollout_timing.py || exit $?
  for lib in build_variants/libfenv_pol_*.so; do
    echo "policy $lib:"; FENV_LIB_OVERRIDE=$PWD/$lib timeout -k 10 90 python tools/rollout_timing.py || exit $?
  done
done
