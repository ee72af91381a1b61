#!/bin/bash
# Round 4: where the MT19937-mode time per reset event goes at config 3.  (1) rates: in-tree
# (draw-ahead) vs build_variants/libfenv_sidecopy.so (the staging copy on a side stream);
# (2) a kernel trace of the in-tree MT run across two events (device gaps, staging copy, launches).
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4n; mkdir -p "$O"; cd "$R"
timeout -k 10 200 python tools/mt_mode_rate.py 1048576 3010 mt19937,philox > "$O/rate_intree.jsonl" 2> "$O/rate_intree.err" &&
FENV_LIB_OVERRIDE=$R/build_variants/libfenv_sidecopy.so timeout -k 10 200 python tools/mt_mode_rate.py 1048576 3010 mt19937 \
  > "$O/rate_sidecopy.jsonl" 2> "$O/rate_sidecopy.err" &&
cat "$O/rate_intree.jsonl" "$O/rate_sidecopy.jsonl" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/trace_mt" -o t \
  -- python3 "$R/tools/mt_mode_rate.py" 1048576 2100 mt19937 > "$O/mt_traced.jsonl" 2> "$O/mt_traced.err"
rc=$?; cat "$O/mt_traced.jsonl"; exit $rc
