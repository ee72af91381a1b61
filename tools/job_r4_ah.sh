#!/bin/bash
# Round 4: the per-sample loss terms formed in the heads phase (FENV_PPO_LOSS_IN_HEADS, "lh":
# no loss phase or barrier) vs in-tree: bit comparison of two updates, PPO tests on lh, phase
# profiles, interleaved timings x4.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4ah; mkdir -p "$O"; cd "$R"
BV=$R/build_variants
timeout -k 10 200 python tools/ppo_params_dump.py "$O/base.npz" > "$O/dump.txt" 2>&1 || exit 1
FENV_LIB_OVERRIDE=$BV/libfenv_lh.so timeout -k 10 200 python tools/ppo_params_dump.py "$O/lh.npz" >> "$O/dump.txt" 2>&1 || exit 1
python tools/ppo_params_dump.py --cmp "$O/base.npz" "$O/lh.npz" | tee "$O/bitcmp.txt"
FENV_LIB_OVERRIDE=$BV/libfenv_lh.so timeout -k 10 500 python -u -m pytest tests/test_gpu_ppo_dp.py tests/test_gpu_rollout.py -m gpu -q -s \
  --timeout 300 --timeout-method thread > "$O/pytest_lh.log" 2>&1
echo "lh tests rc=$?"; tail -2 "$O/pytest_lh.log"; grep "reference-config update" "$O/pytest_lh.log"
for v in p1lh p2lh; do
  echo "== $v" >> "$O/phase.txt"
  FENV_LIB_OVERRIDE=$BV/libfenv_$v.so timeout -k 10 200 python tools/ppo_phase_profile.py >> "$O/phase.txt" 2>> "$O/err.txt" || exit 1
done
cat "$O/phase.txt"
PAIRS=4 VARIANTS="lh" timeout -k 10 600 bash tools/ppo_variant_ab.sh > "$O/ab.txt" 2>> "$O/err.txt"
echo "ab rc=$?"
