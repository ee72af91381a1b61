#!/bin/bash
# GPU-box check: smoke -> parity tests -> short bench.  Each GPU step has its own time limit;
# a crash/abort/timeout stops the script (no further GPU work), a plain test failure does not.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 MPLBACKEND=Agg
stop_if_fatal() {  # $1 = rc, $2 = log
  local rc=$1
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "FATAL rc=$rc in $2"; exit "$rc"; fi
  if grep -q "Timeout" "$2" 2>/dev/null; then echo "TIMEOUT in $2"; exit 124; fi
}
PYTEST_ARGS=${PYTEST_ARGS:-"tests -m gpu -x -v"}
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; stop_if_fatal $rc gpurun_out/smoke.log
timeout -k 10 900 python -u -m pytest $PYTEST_ARGS --timeout 150 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; stop_if_fatal $rc gpurun_out/pytest_gpu.log
if [ -n "${BENCH_ARGS+x}" ]; then
  timeout -k 10 300 python bench.py $BENCH_ARGS > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
fi
