#!/bin/bash
# One GPU call for a round's evidence: GPU tests, smoke(), the driver's bench command, the default bench,
# a rocprofv3 kernel-trace/stats profile of the driver's command, and the two PMC traffic passes.
# Each GPU step has its own time limit; any failure other than a plain test failure stops it.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
TAG=${TAG:-r2}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
export PYTHONUNBUFFERED=1 MPLBACKEND=Agg
fatal() { echo "FATAL rc=$1 at $2"; exit "$1"; }
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread \
    > "$O/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 "$O/pytest_gpu.log"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || fatal $rc pytest
fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke: ok')" > "$O/smoke.log" 2>&1 \
  || fatal $? smoke
echo "smoke ok"
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_driver.json" 2> "$O/bench_driver.err" || fatal $? bench_driver
echo "bench(driver cmd):"; cat "$O/bench_driver.json" | cut -c1-900
if [ -z "${SKIP_DEFAULT:-}" ]; then
  timeout -k 10 300 python bench.py > "$O/bench_default.json" 2> "$O/bench_default.err" || fatal $? bench_default
  echo "bench(default) done"
fi
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/pmc_${TAG}_$C" -o pmc \
    -- python3 "$R/bench.py" --steps 200 --warmup 20 --prewarm-ms 50 --no-cpu-baseline --no-stats --no-policy --no-configs \
    > "$O/pmc_$C.log" 2>&1 || fatal $? "pmc $C"
  echo "pmc $C ok"
done
python3 "$R/tools/pmc_summary.py" "$R/gpurun_out" "$TAG" > "$O/pmc_summary.txt" 2>&1; echo "pmc summary rc=$?"
# Last: rocprofv3 (ROCm 7.2) segfaults inside exit(), after its output is written, when the
# profiled process made a cooperative launch (the PPO update's split launch; DESIGN §9.4,
# profiles/r4_rocprof_coop_exit/), so nothing may follow it in this call.
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_driver" -o bench \
  -- python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 > "$O/bench_driver_under_rocprof.json" 2> "$O/prof_driver.err" \
  || fatal $? rocprof
echo "rocprof ok"
