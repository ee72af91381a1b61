#!/bin/bash
# Round-3 GPU call: config-1 three-role split A/B (build_variants s3 = FENV_SPLIT3 on, s2 = off),
# role attribution (config1_probe) for both, then the GPU suite on the in-tree build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
PARITY_LIBS="build_variants/libfenv_s3.so" ROUNDS=3 timeout -k 10 500 bash tools/env_cfg_ab.sh 2>&1 | grep -v amdgpu.ids || exit $?
for v in s3 s2; do
  echo "== config1_probe $v"
  FENV_LIB_OVERRIDE=$PWD/build_variants/libfenv_$v.so timeout -k 10 120 python -u tools/config1_probe.py 2>&1 | grep -v amdgpu.ids || exit $?
done
TAG=${TAG:-r3s} bash tools/job_r3_suite.sh
