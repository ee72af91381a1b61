#!/bin/bash
# Round 4: MT19937-mode rate at config 3, staging copy on the launch stream (in-tree) vs on a
# side stream (build_variants/libfenv_sidecopy.so), interleaved twice.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4p; mkdir -p "$O"; cd "$R"
for k in 1 2; do
  timeout -k 10 200 python tools/mt_mode_rate.py 1048576 3010 mt19937 >> "$O/rate_intree.jsonl" 2>> "$O/rate.err" || exit 1
  FENV_LIB_OVERRIDE=$R/build_variants/libfenv_sidecopy.so timeout -k 10 200 python tools/mt_mode_rate.py 1048576 3010 mt19937 \
    >> "$O/rate_sidecopy.jsonl" 2>> "$O/rate.err" || exit 1
done
cat "$O/rate_intree.jsonl" "$O/rate_sidecopy.jsonl"
