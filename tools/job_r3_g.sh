#!/bin/bash
# Round-3 GPU call: PPO numerics probe (torch, in-tree, ta0), the PPO A/B, then the GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
VARIANTS="ta0 old" bash tools/job_r3_refcfg.sh || exit $?
PAIRS=2 VARIANTS="ta0 old" timeout -k 10 400 bash tools/ppo_variant_ab.sh 2>&1 | grep -v amdgpu.ids | sed -E "s/'note': [^}]*//; s/'workload': [^,]*,//; s/'samples_per_s'.*//" || exit $?
echo "== PPO phase profile nprof1"
FENV_LIB_OVERRIDE=$PWD/build_variants/libfenv_nprof1.so timeout -k 10 100 python -u tools/ppo_phase_profile.py 2>&1 | grep -v amdgpu.ids || exit $?
TAG=${TAG:-r3g} bash tools/job_r3_suite.sh
grep -E "reference-config|losses torch|       fused" gpurun_out/r3_pytest_gpu_${TAG:-r3g}.log | head -4
