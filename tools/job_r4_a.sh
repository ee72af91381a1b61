#!/bin/bash
# Round 4, first GPU job: the new staging / Philox / lifecycle tests, then the PPO log_std probe.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r4a
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_lifecycle.py \
  "tests/test_gpu_parity.py::test_philox_reset_draws_match_restatement" \
  "tests/test_gpu_parity.py::test_metrics_and_partials" \
  "tests/test_gpu_fullsize.py::test_bench_workload_staggered_resets_vs_oracle" \
  > gpurun_out/r4a/pytest_new.log 2>&1
rc=$?
tail -30 gpurun_out/r4a/pytest_new.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/ppo_logstd_probe.py > gpurun_out/r4a/ppo_logstd_probe.json 2> gpurun_out/r4a/ppo_logstd_probe.err
rc=$?
tail -60 gpurun_out/r4a/ppo_logstd_probe.json
exit $rc
