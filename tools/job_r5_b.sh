#!/bin/bash
# round 5: kernel-trace timelines of bench's timed region at 131072 and 1048576 formations
# (where does the fixed overhead sit?), then the minimal cooperative-launch exit repro
# (tools/coop_exit_min.hip): without the profiler, plain under rocprofv3, and -- last, since it
# may end in the profiler's exit-time SIGSEGV -- cooperative under rocprofv3.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/r5
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for F in 131072 1048576; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$O/trace_$F" -o t \
    -- python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --formations $F --no-policy --no-configs \
    --no-cpu-baseline > "$O/trace_$F.json" 2> "$O/trace_$F.err" || { echo "trace $F rc=$?"; exit 1; }
  echo "trace $F ok"
done
timeout -k 10 60 "$R/tools/coop_exit_min" plain > $O/min_plain.out 2>&1; echo "min plain rc=$?"
timeout -k 10 60 "$R/tools/coop_exit_min" coop > $O/min_coop.out 2>&1; echo "min coop rc=$?"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/min_prof_plain" -o p \
  -- "$R/tools/coop_exit_min" plain > $O/min_prof_plain.out 2> $O/min_prof_plain.err
rc=$?; echo "min plain under rocprofv3 rc=$rc"; [ $rc -eq 0 ] || exit 0
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/min_prof_coop" -o p \
  -- "$R/tools/coop_exit_min" coop > $O/min_prof_coop.out 2> $O/min_prof_coop.err
echo "min coop under rocprofv3 rc=$?"
exit 0
