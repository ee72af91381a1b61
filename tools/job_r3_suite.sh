#!/bin/bash
# Round-3 GPU call: the whole GPU suite (no -x), smoke, the driver's bench command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-suite}
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread \
  > gpurun_out/r3_pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r3_pytest_gpu_$TAG.log
grep -E "^FAILED|Error" gpurun_out/r3_pytest_gpu_$TAG.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | grep -v amdgpu.ids | tail -3
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3_bench_$TAG.json 2> gpurun_out/r3_bench_$TAG.err
rc=$?; echo "bench rc=$rc"; python -c "
import json; d=json.loads(open('gpurun_out/r3_bench_$TAG.json').read().strip().splitlines()[-1])
print('value', d['value'], 'frac', d['roofline']['frac'], 'ms', d['ms_per_step'])
for k in ('ppo_update','policy_rollout','env_configs'):
    v=d.get(k); print(k, {kk: v[kk] for kk in list(v)[:6]} if isinstance(v, dict) else v)
"
exit $rc
