#!/bin/bash
# Round-3 GPU call: the full GPU test suite, then (if it ran to completion) a PPO variant A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/r3_pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/r3_pytest_gpu.log
grep -E "FAILED|reference-config|losses torch|       fused|torch 1ulp" gpurun_out/r3_pytest_gpu.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
if [ -n "${PPO_VARIANTS:-}" ]; then
  PAIRS=${PAIRS:-3} VARIANTS="$PPO_VARIANTS" timeout -k 10 600 bash tools/ppo_variant_ab.sh | sed -E "s/'note': [^}]*//"
fi
