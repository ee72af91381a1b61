#!/bin/bash
# rocprofv3 kernel-trace + stats of tools/rollout_timing.py (config 2: policy_forward, the fused
# rollout kernel and the per-step collector), for profiles/.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${TAG:-r1}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/profpol_$TAG" \
  -o pol -- python3 "$R/tools/rollout_timing.py" > "$R/gpurun_out/profpol_$TAG.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; grep -v amdgpu.ids "$R/gpurun_out/profpol_$TAG.log" | grep -v "^W2\|^E2" | head
find "$R/gpurun_out/profpol_$TAG" -name "*stats*"
