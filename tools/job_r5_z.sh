#!/bin/bash
# round 5: host stalls in the region's first HIP calls vs the HIP runtime's kernel-argument
# placement: HIP_FORCE_DEV_KERNARG=0 / 1 / unset, 262,144 formations, 6 interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5z2
mkdir -p $O
run() {
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --formations 262144 --no-policy \
    --no-configs --no-cpu-baseline --trace-host > $O/$1_$2.json 2> $O/$1_$2.err || exit $?
  python3 - $O/$1_$2.json $1 <<'PY'
import json, sys
d = [json.loads(x) for x in open(sys.argv[1]) if x.startswith("{")][-1]
tr = dict((k, v) for k, v in d.get("host_trace_us", []))
print(sys.argv[2], "value %.4e fixed_us %.1f start_event_us %.1f first_launch_us %.1f second_launch_us %.1f" % (
    d["value"], 1e3 * d["fixed_overhead_ms"], tr.get("start event", -1), tr.get("launch 0", -1), tr.get("launch 1", -1)))
PY
}
for r in 1 2 3 4 5 6; do
  run unset $r
  HIP_FORCE_DEV_KERNARG=0 run k0 $r
  HIP_FORCE_DEV_KERNARG=1 run k1 $r
done
