#!/bin/bash
# rocprofv3 PMC passes (one counter group per run, no tracing domains) over a short bench of the
# default workload; tools/pmc_summary.py turns the CSVs into profiles/pmc_traffic.json.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${TAG:-r1}
ARGS=${BENCH_ARGS:---steps 200 --warmup 20 --no-cpu-baseline --no-stats --no-policy --no-configs}
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/pmc_${TAG}_$C" -o pmc \
    -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/pmc_${TAG}_$C.log" 2>&1
  rc=$?; echo "pmc $C rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$R/gpurun_out/pmc_${TAG}_$C.log"; exit $rc; fi
done
python3 "$R/tools/pmc_summary.py" "$R/gpurun_out" "$TAG"
