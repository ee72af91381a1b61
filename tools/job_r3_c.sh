#!/bin/bash
# Round-3 GPU call: suite + smoke + bench, then the PPO phase profile of both blocks and the A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
TAG=${TAG:-r3c} bash tools/job_r3_suite.sh || exit $?
grep -E "reference-config|losses torch|       fused|torch 1ulp" gpurun_out/r3_pytest_gpu_${TAG:-r3c}.log | head -6
for v in nprof1 nprof2; do
  echo "== PPO phase profile $v"
  FENV_LIB_OVERRIDE=$PWD/build_variants/libfenv_$v.so timeout -k 10 100 python -u tools/ppo_phase_profile.py 2>&1 | grep -v amdgpu.ids || exit $?
done
PAIRS=${PAIRS:-2} VARIANTS="${PPO_VARIANTS:-old pk0 tp0 pt0}" timeout -k 10 700 bash tools/ppo_variant_ab.sh 2>&1 | grep -v amdgpu.ids | sed -E "s/'note': [^}]*//; s/'workload': [^,]*,//; s/'samples_per_s'.*//"
