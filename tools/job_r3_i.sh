#!/bin/bash
# Round-3 GPU call: PPO A/B (bias corrections off the critical path), phase profile, GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
PAIRS=3 VARIANTS="${PPO_VARIANTS:-bcw0 old}" timeout -k 10 500 bash tools/ppo_variant_ab.sh 2>&1 | grep -v amdgpu.ids | sed -E "s/'note': [^}]*//; s/'workload': [^,]*,//; s/'samples_per_s'.*//" || exit $?
echo "== PPO phase profile nprof1"
FENV_LIB_OVERRIDE=$PWD/build_variants/libfenv_nprof1.so timeout -k 10 100 python -u tools/ppo_phase_profile.py 2>&1 | grep -v amdgpu.ids || exit $?
TAG=${TAG:-r3i} bash tools/job_r3_suite.sh
grep -E "reference-config|agents wrong|draw set|final px" gpurun_out/r3_pytest_gpu_${TAG:-r3i}.log | head -12
