#!/bin/bash
# Round 4: MT19937-mode rate at config 3: scalar base/size of the staged set laundered too
# (in-tree) vs only the indices (build_variants/libfenv_prevlaunder.so), interleaved; Philox
# alongside as the reference rate; MT GPU tests first.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4s; mkdir -p "$O"; cd "$R"
timeout -k 10 500 python -u -m pytest tests/test_gpu_lifecycle.py tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > "$O/pytest_mt.log" 2>&1
rc=$?; tail -2 "$O/pytest_mt.log"; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  timeout -k 10 200 python tools/mt_mode_rate.py 1048576 3010 mt19937,philox >> "$O/rate_intree.jsonl" 2>> "$O/rate.err" || exit 1
  FENV_LIB_OVERRIDE=$R/build_variants/libfenv_prevlaunder.so timeout -k 10 200 python tools/mt_mode_rate.py 1048576 3010 mt19937 \
    >> "$O/rate_prev.jsonl" 2>> "$O/rate.err" || exit 1
done
cat "$O/rate_intree.jsonl" "$O/rate_prev.jsonl"
