#!/bin/bash
# Round-3 GPU call: the reference-config PPO update's loss means and final log_std for torch and
# for the fused kernel's numeric variants (tools/ppo_refcfg_probe.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
timeout -k 10 120 python -u tools/ppo_refcfg_probe.py torch 2>&1 | grep -v amdgpu.ids || exit $?
timeout -k 10 120 python -u tools/ppo_refcfg_probe.py 2>&1 | grep -v amdgpu.ids || exit $?
for v in ${VARIANTS:-div acc0 fma0 k160 old}; do
  FENV_LIB_OVERRIDE=$PWD/build_variants/libfenv_$v.so timeout -k 10 120 python -u tools/ppo_refcfg_probe.py 2>&1 | grep -v amdgpu.ids || exit $?
done
