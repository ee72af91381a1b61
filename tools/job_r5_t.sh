#!/bin/bash
# round 5: the timed region's start/end events with hipEventDisableSystemFence (device) vs torch's
# default timing events (system): the driver's command, 4 interleaved rounds, secondary lines off.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5t
mkdir -p $O
for r in 1 2 3 4; do
  for v in system device; do
    timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --event-fence $v \
      --no-cpu-baseline --no-policy --no-configs > $O/${v}_$r.json 2> $O/${v}_$r.err || exit $?
    python3 - "$O/${v}_$r.json" "$v" "$r" <<'PY'
import json, sys
d = [json.loads(x) for x in open(sys.argv[1]) if x.startswith("{")][-1]
print(sys.argv[2], sys.argv[3], "value %.4e kernel_value %.4e fixed_overhead_us %.1f frac %.4f"
      % (d["value"], d["kernel_value"], 1e3 * d["fixed_overhead_ms"], d["roofline"]["frac"]))
PY
  done
done
