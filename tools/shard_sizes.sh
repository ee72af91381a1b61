#!/bin/bash
# Per-GPU rate of the env rollout at the shard sizes of a strong-scaled config 3
# (1M formations over 1/2/4/8 GPUs = 1M/512k/256k/128k formations per GPU), one GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for F in 1048576 524288 262144 131072; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-policy --no-configs --formations $F --steps ${STEPS:-3000} --warmup 100 ${ARGS:-} 2>/dev/null |
    python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(f\"F={$F}: {r['avg_kernel_ms']*1e3:.1f} us/launch  frac {r['frac']:.3f}  value {d['value']:.4g}  wall/step {d['ms_per_step']*1e3:.2f} us\")" || exit 1
done
