#!/bin/bash
# round 5: non-temporal stores per output stream in the headline launch: both (base), obs only
# (ntobs: reward / done plain), reward / done only (ntrd: obs plain); bench.py's config-3 line,
# 2,000 steps, 3 interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5r
mkdir -p $O
for r in 1 2 3; do
  for v in base ntobs ntrd; do
    FENV_LIB_OVERRIDE=build_variants/libfenv_$v.so timeout -k 10 150 python bench.py --steps 2000 --warmup 20 \
      --no-policy --no-configs --no-cpu-baseline > $O/${v}_$r.json 2> $O/${v}_$r.err || exit $?
    python3 -c "
import json; d=json.load(open('$O/${v}_$r.json')); r=d['roofline']
print('$v $r', 'avg_kernel_ms %.4f frac %.4f value %.4g' % (r['avg_kernel_ms'], r['frac'], d['value']))"
  done
done
