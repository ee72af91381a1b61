#!/bin/bash
# Round 4: the loss statistics accumulated in LDS doubles (FENV_PPO_ST_LDS, "stl": no
# private scratch) vs in-tree: bit comparison of two updates, PPO tests on stl, phase
# profiles, interleaved timings x4.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4aj; mkdir -p "$O"; cd "$R"
BV=$R/build_variants
timeout -k 10 200 python tools/ppo_params_dump.py "$O/base.npz" > "$O/dump.txt" 2>&1 || exit 1
FENV_LIB_OVERRIDE=$BV/libfenv_stl.so timeout -k 10 200 python tools/ppo_params_dump.py "$O/stl.npz" >> "$O/dump.txt" 2>&1 || exit 1
python tools/ppo_params_dump.py --cmp "$O/base.npz" "$O/stl.npz" | tee "$O/bitcmp.txt"
FENV_LIB_OVERRIDE=$BV/libfenv_stl.so timeout -k 10 500 python -u -m pytest tests/test_gpu_ppo_dp.py tests/test_gpu_rollout.py -m gpu -q -s \
  --timeout 300 --timeout-method thread > "$O/pytest_stl.log" 2>&1
echo "stl tests rc=$?"; tail -2 "$O/pytest_stl.log"; grep "reference-config update" "$O/pytest_stl.log"
for v in p1stl p2stl; do
  echo "== $v" >> "$O/phase.txt"
  FENV_LIB_OVERRIDE=$BV/libfenv_$v.so timeout -k 10 200 python tools/ppo_phase_profile.py >> "$O/phase.txt" 2>> "$O/err.txt" || exit 1
done
cat "$O/phase.txt"
PAIRS=4 VARIANTS="stl" timeout -k 10 600 bash tools/ppo_variant_ab.sh > "$O/ab.txt" 2>> "$O/err.txt"
echo "ab rc=$?"
