#!/bin/bash
# Round 4 PPO A/B: in-tree (loss fused into the heads phase) vs premerge vs the one-workgroup form.
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=gpurun_out/r4i
mkdir -p $O
for rep in 1 2 3; do
  for v in intree premerge unsplit; do
    L=""; [ $v != intree ] && L=$R/build_variants/libfenv_$v.so
    FENV_LIB_OVERRIDE=$L timeout -k 10 120 python -u tools/ppo_mb_time.py >> $O/timing.jsonl 2>> $O/timing.err || exit $?
  done
done
cat $O/timing.jsonl
