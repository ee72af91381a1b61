#!/bin/bash
# round 5: the timed window's fixed cost with and without the stats pipeline, at the 8-way shard
# size (131072 formations), 4 interleaved pairs of processes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5h
mkdir -p $O
for r in 1 2 3 4; do
  for v in stats nostats; do
    X=""; [ $v = nostats ] && X="--no-stats"
    timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --formations 131072 --no-policy \
      --no-configs --no-cpu-baseline $X > $O/${v}_$r.json 2> $O/${v}_$r.err || exit $?
  done
done
for f in $O/*_[1-4].json; do
  python -c "
import json,sys; d=json.load(open('$f')); print('$f'.split('/')[-1], round(d['ms_per_step']*20e3,1), round(d['roofline']['kernel_ms_timed']*1e3,1), round(d['fixed_overhead_ms']*1e3,1))"
done
