#!/bin/bash
# Round 4: PPO update with split-f16 MFMA (three v_mfma_f32_32x32x16_f16 per 16-deep chunk
# instead of eight fp32 32x32x2): build_variants/libfenv_l2f16.so (layer-2 forward only) and
# libfenv_f16all.so (also the W2-gradient and dL/dh1 chains, dL/dz2 scaled by a power of two)
# vs in-tree.  PPO GPU tests on each variant (incl. the reference-config parity test), then
# interleaved timings.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4z; mkdir -p "$O"; cd "$R"
for v in l2f16 f16all; do
  FENV_LIB_OVERRIDE=$R/build_variants/libfenv_$v.so timeout -k 10 500 python -u -m pytest tests/test_gpu_ppo_dp.py tests/test_gpu_rollout.py -m gpu -v \
    --timeout 300 --timeout-method thread > "$O/pytest_$v.log" 2>&1
  echo "$v tests rc=$?"; tail -2 "$O/pytest_$v.log"
done
for k in 1 2 3; do
  timeout -k 10 200 python tools/ppo_mb_time.py >> "$O/times.jsonl" 2>> "$O/err.txt" || exit 1
  for v in l2f16 f16all; do
    FENV_LIB_OVERRIDE=$R/build_variants/libfenv_$v.so timeout -k 10 200 python tools/ppo_mb_time.py >> "$O/times.jsonl" 2>> "$O/err.txt" || exit 1
  done
done
cat "$O/times.jsonl"
