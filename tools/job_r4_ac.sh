#!/bin/bash
# Round 4: (1) the PPO update's 16-wide phases (heads, head gradients, W1 gradients) also on
# split-f16 (v_mfma_f32_16x16x32_f16; build_variants/libfenv_f16x16.so) vs in-tree: PPO / rollout
# GPU tests on the variant (-s: the reference-config margins), interleaved timings x3;
# (2) the phase profile of the in-tree kernel (prof1 actor, prof2 critic).
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4ac; mkdir -p "$O"; cd "$R"
V=$R/build_variants/libfenv_f16x16.so
FENV_LIB_OVERRIDE=$V timeout -k 10 500 python -u -m pytest tests/test_gpu_ppo_dp.py tests/test_gpu_rollout.py -m gpu -v -s \
  --timeout 300 --timeout-method thread > "$O/pytest_variant.log" 2>&1
echo "variant tests rc=$?"; tail -2 "$O/pytest_variant.log"; grep "reference-config update" "$O/pytest_variant.log"
for k in 1 2 3; do
  timeout -k 10 200 python tools/ppo_mb_time.py >> "$O/times.jsonl" 2>> "$O/err.txt" || exit 1
  FENV_LIB_OVERRIDE=$V timeout -k 10 200 python tools/ppo_mb_time.py >> "$O/times.jsonl" 2>> "$O/err.txt" || exit 1
done
cat "$O/times.jsonl"
for v in 1 2; do
  FENV_LIB_OVERRIDE=$R/build_variants/libfenv_prof$v.so timeout -k 10 200 python tools/ppo_phase_profile.py > "$O/phase_prof$v.txt" 2>> "$O/err.txt" || exit 1
done
cat "$O/phase_prof1.txt" "$O/phase_prof2.txt"
