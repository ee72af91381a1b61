#!/bin/bash
# Round 4: diagnose the MT19937 post-reset mismatch (tools/mt_stage_repro.py), then the log_std probe.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r4b
timeout -k 10 300 python -u tools/mt_stage_repro.py > gpurun_out/r4b/mt_stage_repro.jsonl 2> gpurun_out/r4b/mt_stage_repro.err
rc=$?
cat gpurun_out/r4b/mt_stage_repro.jsonl; tail -5 gpurun_out/r4b/mt_stage_repro.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/ppo_logstd_probe.py > gpurun_out/r4b/ppo_logstd_probe.json 2> gpurun_out/r4b/ppo_logstd_probe.err
rc=$?
tail -70 gpurun_out/r4b/ppo_logstd_probe.json; tail -5 gpurun_out/r4b/ppo_logstd_probe.err
exit $rc
