#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for round in 1 2; do
  for lib in build_variants/libfenv_pol_*.so; do
    FENV_LIB_OVERRIDE=$PWD/$lib timeout -k 10 60 python tools/policy_timing.py ${B:-655360} || exit $?
  done
done
