#!/bin/bash
# Round 4: the fused policy rollout with its per-step uniform values reloaded from the kernarg
# segment (build_variants/libfenv_prkarg.so: SGPR spills 107 -> 20) vs in-tree.  Policy parity
# tests on the variant first, then interleaved timings at config 2.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4w; mkdir -p "$O"; cd "$R"
V=$R/build_variants/libfenv_prkarg.so
FENV_LIB_OVERRIDE=$V timeout -k 10 400 python -u -m pytest tests/test_gpu_policy.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > "$O/pytest_variant.log" 2>&1
rc=$?; tail -2 "$O/pytest_variant.log"; [ $rc -eq 0 ] || exit $rc
for k in 1 2 3; do
  timeout -k 10 200 python tools/policy_rollout_time.py >> "$O/times.jsonl" 2>> "$O/err.txt" || exit 1
  FENV_LIB_OVERRIDE=$V timeout -k 10 200 python tools/policy_rollout_time.py >> "$O/times.jsonl" 2>> "$O/err.txt" || exit 1
done
cat "$O/times.jsonl"
