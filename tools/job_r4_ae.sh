#!/bin/bash
# Round 4: the next-next minibatch's global loads (load_rows / perm_rows) moved from the loop head
# into the norm-exchange shadow (build_variants/libfenv_lg2.so) vs in-tree: PPO tests on the
# variant, interleaved timings x3.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4ae; mkdir -p "$O"; cd "$R"
V=$R/build_variants/libfenv_lg2.so
FENV_LIB_OVERRIDE=$V timeout -k 10 500 python -u -m pytest tests/test_gpu_ppo_dp.py tests/test_gpu_rollout.py -m gpu -q -s \
  --timeout 300 --timeout-method thread > "$O/pytest_variant.log" 2>&1
echo "variant tests rc=$?"; tail -2 "$O/pytest_variant.log"; grep "reference-config update" "$O/pytest_variant.log"
for k in 1 2 3; do
  timeout -k 10 200 python tools/ppo_mb_time.py >> "$O/times.jsonl" 2>> "$O/err.txt" || exit 1
  FENV_LIB_OVERRIDE=$V timeout -k 10 200 python tools/ppo_mb_time.py >> "$O/times.jsonl" 2>> "$O/err.txt" || exit 1
done
cat "$O/times.jsonl"
