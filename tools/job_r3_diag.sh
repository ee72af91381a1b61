#!/bin/bash
# Round-3 GPU call: the partial-record diagnosis, the new PPO tests, and the PPO loss A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
timeout -k 10 120 python -u tools/diag_partials.py 5 || exit $?
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_ppo_dp.py \
  tests/test_gpu_parity.py -k "reference_config or lost_exchange or metrics_and_partials or two_updates or fused_update" \
  > gpurun_out/r3_diag_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|passed|failed|reference-config|losses torch|       fused|torch 1ulp" gpurun_out/r3_diag_tests.log | head -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
PAIRS=3 VARIANTS=lossold timeout -k 10 600 bash tools/ppo_variant_ab.sh | sed -E "s/'note': [^}]*//; s/'workload': [^,]*,//"
