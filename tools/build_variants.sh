#!/bin/bash
# A/B builds of libfenv.so from the current sources: build_variants/libfenv_<tag>.so for each
# "tag:flags" argument (e.g. "nosplit:-DFENV_SPLIT=0").  Built here (CPU), shipped with the tree.
set -eu
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R/marl-distributedformation_amd/csrc"
mkdir -p "$R/build_variants"
B="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt -I../../include -Wall -Wno-unused-result"
S="fenv_kernels.hip fenv_large.hip policy_kernels.hip policy_rollout.hip ppo_update.hip fenv_api.cpp"
for v in "$@"; do
  tag=${v%%:*}; flags=${v#*:}
  $B $flags -o "$R/build_variants/libfenv_$tag.so" $S &
done
wait
ls -la "$R/build_variants"
