#!/bin/bash
# Round 4: DPP wave max for the dL/dz2 scale (was six shuffles): PPO GPU tests, timing x3, phase
# profile (actor / critic).
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4ad; mkdir -p "$O"; cd "$R"
timeout -k 10 500 python -u -m pytest tests/test_gpu_ppo_dp.py tests/test_gpu_rollout.py -m gpu -v -s \
  --timeout 300 --timeout-method thread > "$O/pytest_ppo.log" 2>&1
rc=$?; tail -2 "$O/pytest_ppo.log"; grep "reference-config update" "$O/pytest_ppo.log"; [ $rc -eq 0 ] || exit $rc
for k in 1 2 3; do timeout -k 10 200 python tools/ppo_mb_time.py >> "$O/times.jsonl" 2>> "$O/err.txt" || exit 1; done
cat "$O/times.jsonl"
for v in 1 2; do
  FENV_LIB_OVERRIDE=$R/build_variants/libfenv_prof$v.so timeout -k 10 200 python tools/ppo_phase_profile.py > "$O/phase_prof$v.txt" 2>> "$O/err.txt" || exit 1
done
paste "$O/phase_prof1.txt" "$O/phase_prof2.txt"
