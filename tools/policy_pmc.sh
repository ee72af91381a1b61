#!/bin/bash
# rocprofv3: list gfx950 counters, then SQ counter passes over tools/rollout_timing.py (config 2).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$R/gpurun_out/counters_list.txt" 2>&1; echo "list rc=$?"
i=0
for C in ${PMC_SETS:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"}; do :; done
while read -r SET; do
  [ -z "$SET" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $SET --output-format csv -d "$R/gpurun_out/ppmc_$i" -o p \
    -- python3 "$R/tools/rollout_timing.py" > "$R/gpurun_out/ppmc_$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc: $SET"
  if [ $rc -ne 0 ]; then tail -3 "$R/gpurun_out/ppmc_$i.log"; exit $rc; fi
done < "${PMC_FILE:-$R/tools/policy_pmc_sets.txt}"
