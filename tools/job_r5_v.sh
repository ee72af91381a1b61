#!/bin/bash
# round 5: gc.freeze() before the pre-warm (the pre-window collection no longer idles the GPU
# ~40 ms) vs without, the driver's command, 6 interleaved rounds, secondary lines off.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5v
mkdir -p $O
summ() {
python3 - "$1" "$2" "$3" <<'PY'
import json, sys
d = [json.loads(x) for x in open(sys.argv[1]) if x.startswith("{")][-1]
print(sys.argv[2], sys.argv[3], "value %.4e kernel_value %.4e fixed_overhead_us %.1f"
      % (d["value"], d["kernel_value"], 1e3 * d["fixed_overhead_ms"]))
PY
}
for r in 1 2 3 4 5 6; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-policy \
    --no-configs --no-gc-freeze > $O/nofreeze_$r.json 2> $O/nofreeze_$r.err || exit $?
  summ $O/nofreeze_$r.json nofreeze $r
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-policy \
    --no-configs > $O/freeze_$r.json 2> $O/freeze_$r.err || exit $?
  summ $O/freeze_$r.json freeze $r
done
