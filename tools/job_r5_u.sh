#!/bin/bash
# round 5: host wake-up latency of the closing synchronize: the driver's command with the HIP
# runtime's default wait vs ROC_ACTIVE_WAIT_TIMEOUT set (busy-wait before the interrupt wait),
# 4 interleaved rounds, secondary lines off.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5u
mkdir -p $O
summ() {
python3 - "$1" "$2" "$3" <<'PY'
import json, sys
d = [json.loads(x) for x in open(sys.argv[1]) if x.startswith("{")][-1]
print(sys.argv[2], sys.argv[3], "value %.4e kernel_value %.4e fixed_overhead_us %.1f"
      % (d["value"], d["kernel_value"], 1e3 * d["fixed_overhead_ms"]))
PY
}
for r in 1 2 3 4; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-policy \
    --no-configs > $O/default_$r.json 2> $O/default_$r.err || exit $?
  summ $O/default_$r.json default $r
  ROC_ACTIVE_WAIT_TIMEOUT=2000 timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 \
    --no-cpu-baseline --no-policy --no-configs > $O/wait2000_$r.json 2> $O/wait2000_$r.err || exit $?
  summ $O/wait2000_$r.json wait2000 $r
done
