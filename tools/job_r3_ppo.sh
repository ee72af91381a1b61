#!/bin/bash
# Round-3 GPU call: the PPO tests on the in-tree build, its phase profile, then the variant A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_ppo_dp.py \
  tests/test_gpu_rollout.py > gpurun_out/r3_ppo_tests.log 2>&1
rc=$?; echo "ppo tests rc=$rc"; tail -3 gpurun_out/r3_ppo_tests.log
grep -E "FAILED|reference-config|losses torch|       fused|torch 1ulp" gpurun_out/r3_ppo_tests.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for v in 1 2; do
  echo "== PPO phase profile, block $v"
  FENV_LIB_OVERRIDE=$PWD/build_variants/libfenv_nprof$v.so timeout -k 10 100 python -u tools/ppo_phase_profile.py || exit $?
done
PAIRS=${PAIRS:-2} VARIANTS="${PPO_VARIANTS:-old as0 zs0 le0 ex1 ex2 fma}" timeout -k 10 700 bash tools/ppo_variant_ab.sh | sed -E "s/'note': [^}]*//; s/'workload': [^,]*,//"
