#!/bin/bash
# round 5: MT19937-mode rollout with the staged kernel held to 7 waves/SIMD (72 VGPRs) vs the
# compiler's 73 VGPRs / 6 waves: 3 interleaved rounds, config 3, 3,010 steps (three reset events).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5j
mkdir -p $O
for r in 1 2 3; do
  for v in base mt7; do
    FENV_LIB_OVERRIDE=build_variants/libfenv_$v.so timeout -k 10 120 python tools/mt_mode_rate.py 1048576 3010 \
      > $O/${v}_$r.jsonl 2> $O/${v}_$r.err || exit $?
    echo "$v $r: $(tr '\n' ' ' < $O/${v}_$r.jsonl | cut -c1-400)"
  done
done
