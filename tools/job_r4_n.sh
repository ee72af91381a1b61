#!/bin/bash
# Round 4: kernel trace of MT19937-mode rollouts at config 3 across reset events (where does the
# time per event go: device gaps, the staging copy, shorter launches).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4n; mkdir -p "$O"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/trace_mt" -o t \
  -- python3 "$R/tools/mt_mode_rate.py" 1048576 2100 mt19937 > "$O/mt.jsonl" 2> "$O/mt.err"
rc=$?; cat "$O/mt.jsonl"; exit $rc
