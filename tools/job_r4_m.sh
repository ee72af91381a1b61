#!/bin/bash
# Round 4: (1) GPU lifecycle + MT19937 staging tests with the draw-ahead thread; (2) the MT19937-
# mode rollout rate at config 3 against Philox, with the draw-ahead thread (in-tree) and without
# (build_variants/libfenv_syncmt.so = the previous commit); (3) the driver's bench command with
# the numpy-face (PCIe-inclusive) secondary line.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4m; mkdir -p "$O"; cd "$R"
timeout -k 10 500 python -u -m pytest tests/test_gpu_lifecycle.py tests/test_gpu_parity.py -m gpu -x -v \
  --timeout 200 --timeout-method thread > "$O/pytest_mt.log" 2>&1
rc=$?; tail -3 "$O/pytest_mt.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/mt_mode_rate.py > "$O/mt_mode_rate_ahead.jsonl" 2> "$O/mt_mode_rate_ahead.err" &&
FENV_LIB_OVERRIDE=$R/build_variants/libfenv_syncmt.so timeout -k 10 300 python tools/mt_mode_rate.py \
  > "$O/mt_mode_rate_sync.jsonl" 2> "$O/mt_mode_rate_sync.err" &&
cat "$O/mt_mode_rate_ahead.jsonl" "$O/mt_mode_rate_sync.jsonl" &&
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_driver.json" 2> "$O/bench_driver.err"
rc=$?; echo "rc=$rc"; exit $rc
