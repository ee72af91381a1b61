#!/bin/bash
# Round 4: kernel trace of MT19937- vs Philox-mode rollouts at config 3 (same process), after the
# laundering fix: per-launch durations, staging copies and device gaps around reset events.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4r; mkdir -p "$O"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/trace" -o t \
  -- python3 "$R/tools/mt_mode_rate.py" 1048576 2100 philox,mt19937 > "$O/rate.jsonl" 2> "$O/rate.err"
rc=$?; cat "$O/rate.jsonl"; exit $rc
