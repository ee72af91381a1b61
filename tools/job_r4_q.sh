#!/bin/bash
# Round 4: MT19937 replay with AVX2 clones: GPU MT tests, then the MT-mode rate at config 3 (x2).
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4q; mkdir -p "$O"; cd "$R"
grep -o -m1 "avx2" /proc/cpuinfo > "$O/cpu_avx2.txt"; lscpu > "$O/lscpu.txt" 2>&1
timeout -k 10 500 python -u -m pytest tests/test_gpu_lifecycle.py tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > "$O/pytest_mt.log" 2>&1
rc=$?; tail -2 "$O/pytest_mt.log"; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  timeout -k 10 200 python tools/mt_mode_rate.py 1048576 3010 mt19937,philox >> "$O/rate.jsonl" 2>> "$O/rate.err" || exit 1
done
cat "$O/rate.jsonl"
