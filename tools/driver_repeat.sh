#!/bin/bash
# The driver's bench command, REPS times on one box: steps/warmup honoured, ms_per_step vs the
# kernel time per step, roofline fraction.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2
for i in $(seq 1 ${REPS:-3}); do
  timeout -k 10 200 python bench.py --gpus 1 --steps ${STEPS:-20} --warmup ${WARM:-5} ${ARGS:-} \
    > gpurun_out/r2/driver_rep.json 2> gpurun_out/r2/driver_rep.err || exit $?
  python3 -c "
import json; d=json.load(open('gpurun_out/r2/driver_rep.json')); r=d['roofline']
print('rep $i steps', d['steps'], 'warmup', d['warmup'], 'ms/step %.5f' % d['ms_per_step'],
      'kernel/T %.5f' % (r['avg_kernel_ms'] / d['config']['rollout_chunk']),
      'ratio %.3f' % (d['ms_per_step'] * d['config']['rollout_chunk'] / r['avg_kernel_ms']),
      'frac %.3f' % r['frac'], 'issue_ms %.3f' % d['host_issue_ms'], 'value %.3e' % d['value'])"
done
