#!/bin/bash
# Round 4: ONE PMC pass (set $1 of tools/policy_pmc_sets.txt) over bench.ppo_update_bench at HEAD.
# One pass per call: rocprofv3 segfaults in exit() after writing its output when the profiled
# process made a cooperative launch, so nothing may follow it.
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
SET=$(sed -n "${1}p" "$R/tools/policy_pmc_sets.txt")
timeout -s KILL 150 rocprofv3 --pmc $SET --output-format csv -d "$R/gpurun_out/ppopmc_$1" -o pmc \
  -- python3 "$R/tools/ppo_pmc_run.py" > "$R/gpurun_out/ppo_pmc_$1.log" 2>&1
rc=$?; echo "pass $1 rc=$rc"; ls "$R/gpurun_out/ppopmc_$1"; exit 0
