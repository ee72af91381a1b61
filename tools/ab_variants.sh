#!/bin/bash
# A/B the build_variants/libfenv_*.so builds on the default bench workload, two rounds each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for round in 1 2; do
  for lib in build_variants/libfenv_*.so; do
    FENV_LIB_OVERRIDE=$PWD/$lib timeout -k 10 120 python bench.py --steps 3000 --warmup 200 --no-cpu-baseline --no-policy --no-configs ${AB_ARGS:-} > gpurun_out/ab.json 2>gpurun_out/ab.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "FAIL $lib rc=$rc"; tail -3 gpurun_out/ab.err; exit $rc; fi
    python -c "import json;d=json.load(open('gpurun_out/ab.json'));r=d['roofline'];print('$round','$lib','%.4g'%d['value'],'kern_ms=%.4f'%r['avg_kernel_ms'],'frac=%.3f'%r['frac'])"
  done
done
