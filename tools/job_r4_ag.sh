#!/bin/bash
# Round 4: in-tree with the loss constants in the heads phase, the ratio on hardware exp2 and the
# late loss sums (FENV_PPO_LC_EARLY / HWEXP / SUMS_LATE = 1) vs build_variants/libfenv_prev.so
# (the previous HEAD's kernel): full GPU suite, phase profiles, interleaved timings x4.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4ag; mkdir -p "$O"; cd "$R"
BV=$R/build_variants
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -s > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$O/pytest_gpu.log"; grep "reference-config update" "$O/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
for v in p1 prof2; do
  echo "== $v" >> "$O/phase.txt"
  FENV_LIB_OVERRIDE=$BV/libfenv_$v.so timeout -k 10 200 python tools/ppo_phase_profile.py >> "$O/phase.txt" 2>> "$O/err.txt" || exit 1
done
cat "$O/phase.txt"
PAIRS=4 VARIANTS="prev" timeout -k 10 600 bash tools/ppo_variant_ab.sh > "$O/ab.txt" 2>> "$O/err.txt"
echo "ab rc=$?"
