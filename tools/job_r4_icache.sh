#!/bin/bash
# Round 4: instruction-cache counters over the fused PPO update (one PMC pass; nothing may follow
# it, see tools/job_r4_ppopmc.sh): is the ~1k-cycle loop-head ("gather") phase i-cache misses?
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVES SQ_BUSY_CYCLES \
  --output-format csv -d "$R/gpurun_out/ppo_icache" -o pmc \
  -- python3 "$R/tools/ppo_pmc_run.py" > "$R/gpurun_out/ppo_icache.log" 2>&1
rc=$?; echo "icache pass rc=$rc"; ls "$R/gpurun_out/ppo_icache"; exit 0
