#!/bin/bash
# Same-box A/B of the fused PPO update: the in-tree libfenv.so ("base") vs
# build_variants/libfenv_<v>.so for v in VARIANTS, interleaved, PAIRS rounds; prints bench.py's
# ppo_update line (ms per update, us per minibatch) per run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PAIRS=${PAIRS:-3}
VARIANTS=${VARIANTS:-latepg}
run() {
  timeout -k 10 120 python -c "import sys; sys.argv=['x']; import bench, torch, pkgload; \
pkg = pkgload.load(); print('$1', bench.ppo_update_bench(pkg.__name__, torch.device('cuda', 0)), flush=True)"
}
for k in $(seq "$PAIRS"); do
  run base || exit $?
  for v in $VARIANTS; do
    FENV_LIB_OVERRIDE=$PWD/build_variants/libfenv_$v.so run $v || exit $?
  done
done
