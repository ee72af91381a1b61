#!/bin/bash
# round 5: host-issue spikes at the start of the timed region: a 500 us sleep + stream query
# before t0 (settle) vs none, 262,144 formations, --trace-host, 8 interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5y
mkdir -p $O
for r in 1 2 3 4 5 6 7 8; do
  for v in 0 500; do
    timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --formations 262144 --no-policy \
      --no-configs --no-cpu-baseline --trace-host --settle-us $v > $O/s${v}_$r.json 2> $O/s${v}_$r.err || exit $?
    python3 - $O/s${v}_$r.json $v <<'PY'
import json, sys
d = [json.loads(x) for x in open(sys.argv[1]) if x.startswith("{")][-1]
tr = dict((k, v) for k, v in d.get("host_trace_us", []))
print("settle", sys.argv[2], "value %.4e kv %.4e fixed_us %.1f start_event_us %.1f first_launch_us %.1f" % (
    d["value"], d["kernel_value"], 1e3 * d["fixed_overhead_ms"], tr.get("start event", -1), tr.get("launch 0", -1)))
PY
  done
done
