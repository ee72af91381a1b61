#!/bin/bash
# Round 4: the heads (mu, value) on VALU fma chains + a DPP quad sum instead of 16 16x16x4 MFMAs
# with 2 resp. 1 real output columns (FENV_PPO_HEADS_VALU, "hv") vs in-tree: PPO tests on hv,
# actor phase profile, interleaved timings x4.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4ai; mkdir -p "$O"; cd "$R"
BV=$R/build_variants
FENV_LIB_OVERRIDE=$BV/libfenv_hv.so timeout -k 10 500 python -u -m pytest tests/test_gpu_ppo_dp.py tests/test_gpu_rollout.py -m gpu -q -s \
  --timeout 300 --timeout-method thread > "$O/pytest_hv.log" 2>&1
echo "hv tests rc=$?"; tail -2 "$O/pytest_hv.log"; grep "reference-config update" "$O/pytest_hv.log"
echo "== p1hv" >> "$O/phase.txt"
FENV_LIB_OVERRIDE=$BV/libfenv_p1hv.so timeout -k 10 200 python tools/ppo_phase_profile.py >> "$O/phase.txt" 2>> "$O/err.txt" || exit 1
cat "$O/phase.txt"
PAIRS=4 VARIANTS="hv" timeout -k 10 600 bash tools/ppo_variant_ab.sh > "$O/ab.txt" 2>> "$O/err.txt"
echo "ab rc=$?"
