#!/bin/bash
# Same-box A/B of the env step kernel: bench.py (env only) with the in-tree library and with
# every build_variants/libfenv_*.so, two rounds.  Prints avg kernel ms and the HBM fraction.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
run() {
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-policy --no-configs --steps ${STEPS:-2000} --warmup 100 ${ARGS:-} 2>/dev/null |
    python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(f\"{r['avg_kernel_ms']*1e3:.1f} us  {r['achieved']:.0f} GB/s  frac {r['frac']:.3f}  value {d['value']:.4g}\")"
}
for round in $(seq 1 ${ROUNDS:-2}); do
  echo "in-tree: $(run)" || exit 1
  for lib in build_variants/libfenv_*.so; do
    [ -e "$lib" ] || continue
    echo "$lib: $(FENV_LIB_OVERRIDE=$PWD/$lib run)" || exit 1
  done
done
