#!/bin/bash
# Round 4: Adam-rate fix A/B -- whole-step bias vs float64 along the reference trajectory
# (tools/ppo_step_probe.py), one reference-config update's loss means, us per minibatch.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r4e
mkdir -p $O
for v in adamold adamfix; do
  FENV_LIB_OVERRIDE=$PWD/build_variants/libfenv_$v.so timeout -k 10 300 python -u tools/ppo_step_probe.py > $O/step_$v.json 2> $O/step_$v.err || exit $?
done
for v in adamold adamfix adamfix_tacc; do
  FENV_LIB_OVERRIDE=$PWD/build_variants/libfenv_$v.so timeout -k 10 120 python -u tools/ppo_refcfg_probe.py > $O/refcfg_$v.txt 2>&1 || exit $?
done
for rep in 1 2; do
  for v in adamold adamfix adamfix_tacc; do
    FENV_LIB_OVERRIDE=$PWD/build_variants/libfenv_$v.so timeout -k 10 120 python -u tools/ppo_mb_time.py >> $O/timing.jsonl 2> $O/timing.err || exit $?
  done
done
cat $O/refcfg_*.txt | grep -v amdgpu.ids; cat $O/timing.jsonl
for v in adamold adamfix; do python3 -c "
import json; d=json.load(open('$O/step_$v.json')); print('$v', 'all', d['all']); [print('   ', k, {w: (round(x['mean'],9), round(x['rms'],7)) for w,x in g.items()}) for k,g in d['groups'].items()]"; done
