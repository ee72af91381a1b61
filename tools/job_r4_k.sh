#!/bin/bash
# Round 4: (1) the headline PMC traffic passes at HEAD (bench --no-policy: no PPO launch);
# (2) rocprofv3 on the PPO update with the split launch made a plain (non-cooperative) launch
# (build_variants/libfenv_nocoop.so): if this exits cleanly, the exit-time SIGSEGV of
# gpurun_out/r4j/ppo.err comes from profiling a cooperative launch.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4k; mkdir -p "$O"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/pmc_r4_$C" -o pmc \
    -- python3 "$R/bench.py" --steps 200 --warmup 20 --prewarm-ms 50 --no-cpu-baseline --no-stats --no-policy --no-configs \
    > "$O/pmc_$C.log" 2>&1 || { echo "pmc $C rc=$?"; exit 1; }
  echo "pmc $C ok"
done
python3 "$R/tools/pmc_summary.py" "$R/gpurun_out" r4 > "$O/pmc_summary.txt" 2>&1; echo "pmc summary rc=$?"
FENV_LIB_OVERRIDE=$R/build_variants/libfenv_nocoop.so timeout -k 10 300 rocprofv3 --kernel-trace --stats \
  --output-format csv -d "$O/prof_ppo_nocoop" -o p -- python3 "$R/tools/ppo_mb_time.py" \
  > "$O/ppo_nocoop.json" 2> "$O/ppo_nocoop.err"
rc=$?; echo "ppo nocoop under rocprof rc=$rc"; exit $rc
