#!/bin/bash
# Round-3 GPU call: the partial-record diagnosis, the whole GPU suite (no -x), the driver's bench,
# the PPO phase profile of both blocks.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u tools/diag_partials2.py > gpurun_out/r3_diag2.log 2>&1
rc=$?; echo "diag2 rc=$rc"; cat gpurun_out/r3_diag2.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread \
  > gpurun_out/r3_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r3_pytest_gpu.log
grep -E "FAILED|Error" gpurun_out/r3_pytest_gpu.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err
rc=$?; echo "bench rc=$rc"; head -c 1500 gpurun_out/r3_bench.json
[ $rc -eq 0 ] || exit $rc
for v in 1 2; do
  echo "== PPO phase profile, block $v"
  FENV_LIB_OVERRIDE=$PWD/build_variants/libfenv_prof$v.so timeout -k 10 100 python -u tools/ppo_phase_profile.py || exit $?
done
