#!/bin/bash
# Same-box A/B of fused PPO update builds: the in-tree libfenv.so and every
# build_variants/libfenv_*.so whose name does not end in "p" (those are -DFENV_PPO_PROFILE=1
# builds: their per-phase cycle profile is printed once each), interleaved over ROUNDS rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
run() {
  timeout -k 10 120 python -c "import sys; sys.argv=['x']; import bench, torch, pkgload; \
pkg = pkgload.load(); r = bench.ppo_update_bench(pkg.__name__, torch.device('cuda', 0)); \
print(f\"{'$1':12s} {r['ms_per_update']:8.2f} ms/update  {r['us_per_minibatch']:6.2f} us/minibatch\", flush=True)" 2>/dev/null
}
for lib in build_variants/libfenv_*p.so; do
  [ -e "$lib" ] || continue
  echo "== phase profile $(basename "$lib")"
  FENV_LIB_OVERRIDE=$PWD/$lib timeout -k 10 120 python tools/ppo_phase_profile.py 2>/dev/null || exit 1
done
for round in $(seq 1 "${ROUNDS:-3}"); do
  run in-tree || exit 1
  for lib in build_variants/libfenv_*.so; do
    case "$lib" in *p.so) continue ;; esac
    n=$(basename "$lib" .so); FENV_LIB_OVERRIDE=$PWD/$lib run "${n#libfenv_}" || exit 1
  done
done
