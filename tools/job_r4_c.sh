#!/bin/bash
# Round 4: MT19937 post-reset failure -- repro before (idle-lane terminal stores ungated,
# build_variants/libfenv_nolive.so) and after (in-tree) the fix, then the new GPU tests.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r4c
FENV_LIB_OVERRIDE=$PWD/build_variants/libfenv_nolive.so timeout -k 10 300 python -u tools/mt_stage_repro.py \
  > gpurun_out/r4c/mt_stage_repro_before.jsonl 2> gpurun_out/r4c/mt_stage_repro_before.err || exit $?
timeout -k 10 300 python -u tools/mt_stage_repro.py \
  > gpurun_out/r4c/mt_stage_repro_after.jsonl 2> gpurun_out/r4c/mt_stage_repro_after.err || exit $?
cat gpurun_out/r4c/mt_stage_repro_before.jsonl gpurun_out/r4c/mt_stage_repro_after.jsonl
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_lifecycle.py \
  "tests/test_gpu_parity.py::test_idle_lanes_store_no_terminal_state" \
  "tests/test_gpu_parity.py::test_philox_reset_draws_match_restatement" \
  "tests/test_gpu_parity.py::test_metrics_and_partials" \
  "tests/test_gpu_fullsize.py::test_bench_workload_staggered_resets_vs_oracle" \
  > gpurun_out/r4c/pytest_new.log 2>&1
rc=$?
tail -40 gpurun_out/r4c/pytest_new.log
exit $rc
