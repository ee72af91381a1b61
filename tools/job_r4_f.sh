#!/bin/bash
# Round 4: the PPO test file (reference-config parity, step bias, lost exchange under the
# cooperative launch), PPO timing, and the whole-trajectory step probe of the final build.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_ppo_dp.py \
  > $O/pytest_ppo.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|reference-config|losses torch|fused \{|1ulp" $O/pytest_ppo.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do timeout -k 10 120 python -u tools/ppo_mb_time.py >> $O/timing.jsonl 2>> $O/timing.err || exit $?; done
cat $O/timing.jsonl
timeout -k 10 300 python -u tools/ppo_step_probe.py > $O/step_probe.json 2> $O/step_probe.err || exit $?
python3 -c "import json; d=json.load(open('$O/step_probe.json')); print(d['all'])"
