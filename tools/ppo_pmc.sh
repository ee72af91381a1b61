#!/bin/bash
# SQ / GRBM PMC passes (tools/policy_pmc_sets.txt, one rocprofv3 run per set) over one
# bench.ppo_update_bench run -> profiles-ready JSON for k_ppo_update (tools/policy_pmc_summary.py).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
i=0
while read -r set; do
  i=$((i + 1))
  timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d "$R/gpurun_out/ppopmc_$i" -o pmc \
    -- python3 "$R/tools/ppo_pmc_run.py" > "$R/gpurun_out/ppo_pmc_$i.log" 2>&1 || { echo "pass $i rc=$?"; exit 1; }
  echo "pass $i ok: $(tail -n 1 "$R/gpurun_out/ppo_pmc_$i.log" | cut -c1-200)"
done < "$R/tools/policy_pmc_sets.txt"
python3 "$R/tools/policy_pmc_summary.py" "$R/gpurun_out" "$R/gpurun_out/r3_ppo_pmc_sq.json" k_ppo_update ppopmc_ \
  "tools/ppo_pmc.sh) over bench.ppo_update_bench, 1000 x 5, n_steps 10, batch 64, 10 epochs"
