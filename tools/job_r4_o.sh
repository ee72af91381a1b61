#!/bin/bash
# Round 4: MT19937 kernels with the reset branch's indices laundered (no hoisted addresses: the
# config-3 kernel back to 6 waves/SIMD).  GPU suite subset for the MT paths, then the MT-mode
# rate at config 3 against Philox (in-tree) and against the previous build (libfenv_syncmt.so).
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4o; mkdir -p "$O"; cd "$R"
timeout -k 10 500 python -u -m pytest tests/test_gpu_lifecycle.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -v \
  --timeout 200 --timeout-method thread > "$O/pytest_mt.log" 2>&1
rc=$?; tail -3 "$O/pytest_mt.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/mt_mode_rate.py 1048576 3010 mt19937,philox > "$O/rate_intree.jsonl" 2> "$O/rate_intree.err" &&
FENV_LIB_OVERRIDE=$R/build_variants/libfenv_syncmt.so timeout -k 10 200 python tools/mt_mode_rate.py 1048576 3010 mt19937 \
  > "$O/rate_syncmt.jsonl" 2> "$O/rate_syncmt.err"
rc=$?; cat "$O/rate_intree.jsonl" "$O/rate_syncmt.jsonl"; exit $rc
