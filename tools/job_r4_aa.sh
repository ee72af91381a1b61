#!/bin/bash
# Round 4: the split-f16 PPO update in-tree.  (1) the PPO / rollout GPU tests (-s: the reference-
# config test prints its margins); (2) the reference-config probe and the per-step bias probe
# vs float64; (3) us per minibatch x3; (4) the whole GPU suite.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4aa; mkdir -p "$O"; cd "$R"
timeout -k 10 500 python -u -m pytest tests/test_gpu_ppo_dp.py tests/test_gpu_rollout.py -m gpu -v -s \
  --timeout 300 --timeout-method thread > "$O/pytest_ppo.log" 2>&1
rc=$?; tail -2 "$O/pytest_ppo.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ppo_refcfg_probe.py > "$O/refcfg.txt" 2> "$O/refcfg.err" || exit 1
timeout -k 10 600 python tools/ppo_step_probe.py > "$O/step_probe.json" 2> "$O/step_probe.err" || exit 1
for k in 1 2 3; do timeout -k 10 200 python tools/ppo_mb_time.py >> "$O/times.jsonl" 2>> "$O/err.txt" || exit 1; done
cat "$O/times.jsonl"; tail -5 "$O/refcfg.txt"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$O/pytest_gpu.log"; exit $rc
