#!/bin/bash
# Round-3 GPU call: suite + smoke + bench, then the PPO phase profile (new / old) and the A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
TAG=${TAG:-r3b} bash tools/job_r3_suite.sh || exit $?
for v in nprof1 prof1; do
  echo "== PPO phase profile $v"
  FENV_LIB_OVERRIDE=$PWD/build_variants/libfenv_$v.so timeout -k 10 100 python -u tools/ppo_phase_profile.py 2>&1 | grep -v amdgpu.ids || exit $?
done
PAIRS=${PAIRS:-2} VARIANTS="${PPO_VARIANTS:-old as0 sp0 ap0 b20 b10 hk0}" timeout -k 10 700 bash tools/ppo_variant_ab.sh 2>&1 | grep -v amdgpu.ids | sed -E "s/'note': [^}]*//; s/'workload': [^,]*,//; s/'samples_per_s'.*//"
