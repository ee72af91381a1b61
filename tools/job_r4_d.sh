#!/bin/bash
# Round 4: PPO precision variants -- per-minibatch gradient error vs float64 along the reference
# trajectory (tools/ppo_logstd_probe.py), the final loss means of one reference-config update
# (tools/ppo_refcfg_probe.py), and us per minibatch, for the in-tree build and three variants.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r4d
mkdir -p $O
V="intree tacc exact lcx"
lib() { [ "$1" = intree ] && echo "" || echo "$PWD/build_variants/libfenv_$1.so"; }
timeout -k 10 120 python -u tools/ppo_refcfg_probe.py torch > $O/refcfg_torch.txt 2>&1 || exit $?
for v in $V; do
  FENV_LIB_OVERRIDE=$(lib $v) timeout -k 10 300 python -u tools/ppo_logstd_probe.py > $O/logstd_$v.json 2> $O/logstd_$v.err || exit $?
  FENV_LIB_OVERRIDE=$(lib $v) timeout -k 10 120 python -u tools/ppo_refcfg_probe.py > $O/refcfg_$v.txt 2>&1 || exit $?
done
for rep in 1 2; do
  for v in $V; do
    FENV_LIB_OVERRIDE=$(lib $v) timeout -k 10 120 python -u tools/ppo_mb_time.py >> $O/timing.jsonl 2> $O/timing.err || exit $?
  done
done
cat $O/refcfg_*.txt | grep -v amdgpu.ids; cat $O/timing.jsonl
for v in $V; do python3 -c "
import json,sys; d=json.load(open('$O/logstd_$v.json')); print('$v', 'log_std k rms', d['log_std']['kernel']['rms'], 't32 rms', d['log_std']['torch32']['rms'], 'groups k/t32 rms', [round(g['k']['rms_err']/max(g['t32']['rms_err'],1e-30),2) for g in d['groups'].values()])"; done
