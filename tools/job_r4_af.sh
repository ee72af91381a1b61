#!/bin/bash
# Round 4: PPO loss-phase variants vs in-tree.  lc = the loss constants in the heads phase
# (FENV_PPO_LC_EARLY), hx = the ratio on hardware exp2 (FENV_PPO_HWEXP), sl = one gradient sum per
# wave and the statistics sums in the exchange shadow (FENV_PPO_SUMS_LATE), all3 = the three.
# PPO tests on all3, phase profiles (actor block p1*, critic block p2*), interleaved timings x3.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4af; mkdir -p "$O"; cd "$R"
BV=$R/build_variants
FENV_LIB_OVERRIDE=$BV/libfenv_all3.so timeout -k 10 500 python -u -m pytest tests/test_gpu_ppo_dp.py tests/test_gpu_rollout.py -m gpu -q -s \
  --timeout 300 --timeout-method thread > "$O/pytest_all3.log" 2>&1
echo "all3 tests rc=$?"; tail -2 "$O/pytest_all3.log"; grep "reference-config update" "$O/pytest_all3.log"
for v in p1 p1lchx p1sl prof2 p2lchx p2sl; do
  echo "== $v" >> "$O/phase.txt"
  FENV_LIB_OVERRIDE=$BV/libfenv_$v.so timeout -k 10 200 python tools/ppo_phase_profile.py >> "$O/phase.txt" 2>> "$O/err.txt" || exit 1
done
cat "$O/phase.txt"
PAIRS=3 VARIANTS="lc hx lchx sl all3" timeout -k 10 800 bash tools/ppo_variant_ab.sh > "$O/ab.txt" 2>> "$O/err.txt"
echo "ab rc=$?"; cat "$O/ab.txt"
