#!/bin/bash
# The driver's short bench command (--steps 20 --warmup 5: two timed launches) with and without
# the stats reduction, in-tree library vs build_variants/libfenv_dpp.so, ROUNDS rounds; prints
# the per-launch times of the timed window.  A variant's parity tests run first (TESTS=0 skips).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-first}
mkdir -p "$O"
V=$PWD/build_variants/libfenv_dpp.so
if [ "${TESTS:-1}" = 1 ]; then
  FENV_LIB_OVERRIDE=$V timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_fullsize.py > "$O/tests_dpp.txt" 2>&1 || { tail -5 "$O/tests_dpp.txt"; exit 1; }
  tail -1 "$O/tests_dpp.txt"
fi
for i in $(seq "${ROUNDS:-3}"); do
  for v in base dpp; do
    for st in s n; do
      extra=""; [ $st = n ] && extra=--no-stats
      if [ $v = dpp ]; then export FENV_LIB_OVERRIDE=$V; else unset FENV_LIB_OVERRIDE; fi
      timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-policy \
        --no-configs $extra > "$O/${v}_${st}$i.json" 2>/dev/null || exit 1
      python3 -c "import json; d=json.load(open('$O/${v}_${st}$i.json')); r=d['roofline']; \
print('$v $st$i', round(r['frac'], 4), [round(x, 4) for x in r['launch_ms_first']], round(d['ms_per_step'], 4))"
    done
  done
done
