#!/bin/bash
# round 5: where the region's host issue time goes when it spikes (~200 us) at 262,144 formations:
# the driver's command with --trace-host, 8 processes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5w
mkdir -p $O
for r in 1 2 3 4 5 6 7 8; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --formations 262144 --no-policy \
    --no-configs --no-cpu-baseline --trace-host > $O/t_$r.json 2> $O/t_$r.err || exit $?
  python3 - $O/t_$r.json <<'PY'
import json, sys
d = [json.loads(x) for x in open(sys.argv[1]) if x.startswith("{")][-1]
print("fixed_us %.1f issue_ms %.3f" % (1e3 * d["fixed_overhead_ms"], d["host_issue_ms"]), json.dumps(d.get("host_trace_us"))[:600])
PY
done
