#!/bin/bash
# Round 4: shader-clock phase profile of the split-f16 PPO update (actor block: prof1, critic: prof2).
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4ab; mkdir -p "$O"; cd "$R"
for v in 1 2; do
  FENV_LIB_OVERRIDE=$R/build_variants/libfenv_prof$v.so timeout -k 10 200 python tools/ppo_phase_profile.py > "$O/phase_prof$v.txt" 2>> "$O/err.txt" || exit 1
done
cat "$O/phase_prof1.txt" "$O/phase_prof2.txt"
