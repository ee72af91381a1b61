#!/bin/bash
# rocprofv3 kernel-trace + stats of the default bench workload (no PMC here; PMC passes are
# separate runs, see tools/gpu_pmc.sh).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${TAG:-r1}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$TAG" \
  -o bench -- python3 "$R/bench.py" ${BENCH_ARGS:---steps 2000 --warmup 100 --no-cpu-baseline --no-policy --no-configs} \
  > "$R/gpurun_out/bench_prof_$TAG.json" 2> "$R/gpurun_out/bench_prof_$TAG.err"
rc=$?; echo "rocprof rc=$rc"; cat "$R/gpurun_out/bench_prof_$TAG.json"
find "$R/gpurun_out/prof_$TAG" -name "*stats*" | head
