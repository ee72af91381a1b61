#!/bin/bash
# Round 4: which part of bench.py makes rocprofv3 --kernel-trace --stats segfault at process exit
# (gpurun_out/r4/prof_driver.err: SIGSEGV inside exit() after the tool's output was written).
# Step 1 profiles bench without the policy / PPO lines, step 2 the PPO update alone (its split
# launch is cooperative since round 4).  Ordered so that the step expected to pass runs first.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4j; mkdir -p "$O"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_nopolicy" -o b \
  -- python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-policy --no-cpu-baseline \
  > "$O/nopolicy.json" 2> "$O/nopolicy.err" && echo "nopolicy ok" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_ppo" -o p \
  -- python3 "$R/tools/ppo_mb_time.py" > "$O/ppo.json" 2> "$O/ppo.err" && echo "ppo ok"
rc=$?; echo "rc=$rc"; exit $rc
