#!/bin/bash
# round 5: MT19937 mode runs its launches without a reset event on the Philox instantiation
# (fenv_api.cpp launch_consts): the GPU suite at the new library, then the rate A/B against HEAD
# (3 interleaved rounds) and one rocprofv3 kernel-stats pass, config 3, 3,010 steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5l
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest exit $?"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for r in 1 2 3; do
  for v in base mtp; do
    FENV_LIB_OVERRIDE=build_variants/libfenv_$v.so timeout -k 10 120 python tools/mt_mode_rate.py 1048576 3010 \
      > $O/${v}_$r.jsonl 2> $O/${v}_$r.err || exit $?
    echo "$v $r: $(tr '\n' ' ' < $O/${v}_$r.jsonl | cut -c1-400)"
  done
done
v=mtp
FENV_LIB_OVERRIDE=build_variants/libfenv_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats \
  --output-format csv -d $O/prof_$v -o p -- python tools/mt_mode_rate.py 1048576 3010 \
  > $O/prof_$v.log 2>&1 || { echo "rocprof $v exit $?"; }
f=$(ls $O/prof_$v/*/p_kernel_stats.csv $O/prof_$v/p_kernel_stats.csv 2>/dev/null | head -1)
[ -n "$f" ] && grep -E "rollout_wave_rs" "$f" | cut -c1-300
exit 0
