#!/bin/bash
# Same-box HBM ceiling vs the headline kernel: ubench_ceiling (copy4 / write4 / the rollout's
# exact byte mix with no arithmetic) interleaved with short headline-only bench runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-ceil}
mkdir -p "$O"
for r in 1 2; do
  timeout -k 10 120 ./tools/ubench_ceiling > "$O/ub$r.txt" 2>&1 || { echo "ubench rc=$?"; exit 1; }
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-policy \
    --no-configs ${BENCH_EXTRA:-} > "$O/b$r.json" 2> "$O/b$r.err" || { echo "bench rc=$?"; exit 1; }
done
cat "$O"/ub*.txt
python3 - "$O" <<'EOF'
import json, sys
for r in (1, 2):
    d = json.load(open(f"{sys.argv[1]}/b{r}.json"))["roofline"]
    print(f"bench {r}: {d['avg_kernel_ms']:.4f} ms/launch  {d['achieved']:.1f} GB/s  frac {d['frac']:.3f}")
EOF
