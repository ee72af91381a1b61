#!/bin/bash
# round 5: MT19937 staging by DMA on the handle's own stream + 4-part parallel host draws + the
# 7-wave MT kernel ("new", in-tree) against the previous HEAD's library ("base"): the MT19937
# parity tests first, then 3 interleaved rounds of tools/mt_mode_rate.py at config 3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5k
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "mt or staging or MT or lifecycle or sharded or reset" > $O/pytest_mt.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_mt.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in base new; do
    FENV_LIB_OVERRIDE=build_variants/libfenv_$v.so timeout -k 10 120 python tools/mt_mode_rate.py 1048576 3010 \
      > $O/${v}_$r.jsonl 2> $O/${v}_$r.err || exit $?
    echo "$v $r: $(python -c "
import json,sys
for l in open('$O/${v}_$r.jsonl'): d=json.loads(l); print(d['mode'], '%.4g' % d['agent_steps_per_s'], 'maxhost %.1f ms' % d['max_host_ms_per_call'], end='; ')")"
  done
done
