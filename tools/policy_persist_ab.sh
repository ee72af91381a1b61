#!/bin/bash
# Fused policy rollout A/B on one box: build_variants/libfenv_pol_*.so interleaved
# (tools/rollout_timing.py, BASELINE config 2), ROUNDS rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for round in $(seq 1 ${ROUNDS:-3}); do
  for lib in build_variants/libfenv_pol_*.so; do
    echo "$lib:"; FENV_LIB_OVERRIDE=$PWD/$lib timeout -k 10 90 python tools/rollout_timing.py 2>/dev/null | grep fused=True || exit $?
  done
done
