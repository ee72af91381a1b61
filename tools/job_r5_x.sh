#!/bin/bash
# round 5: the timed region's start/end events through the HIP C API (ctypes) vs torch.cuda.Event,
# 262,144 formations (the 4-GPU shard of config 3) and 1,048,576, --trace-host, 6 interleaved
# rounds each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5x
mkdir -p $O
for F in 262144 1048576; do
for r in 1 2 3 4 5 6; do
  for v in torch hip; do
    timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --formations $F --no-policy \
      --no-configs --no-cpu-baseline --trace-host --region-events $v > $O/${v}_${F}_$r.json 2> $O/${v}_${F}_$r.err || exit $?
    python3 - $O/${v}_${F}_$r.json $v $F <<'PY'
import json, sys
d = [json.loads(x) for x in open(sys.argv[1]) if x.startswith("{")][-1]
tr = dict((k, v) for k, v in d.get("host_trace_us", []))
print(sys.argv[2], sys.argv[3], "value %.4e kv %.4e fixed_us %.1f issue_ms %.3f first_launch_us %.1f" % (
    d["value"], d["kernel_value"], 1e3 * d["fixed_overhead_ms"], d["host_issue_ms"], tr.get("launch 0", -1)))
PY
  done
done
done
