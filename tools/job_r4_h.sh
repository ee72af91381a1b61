#!/bin/bash
# Round 4: PPO with the loss fused into the heads phase -- the PPO test file, us per minibatch
# against the previous build (r4base), phase profiles; then the policy-rollout PMC passes at HEAD
# and the bench's N > 1 path rehearsed with two gloo ranks on the one GPU.
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=gpurun_out/r4h
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_ppo_dp.py \
  > $O/pytest_ppo.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|reference-config|losses torch|fused \{|1ulp" $O/pytest_ppo.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  timeout -k 10 120 python -u tools/ppo_mb_time.py >> $O/timing.jsonl 2>> $O/timing.err || exit $?
  FENV_LIB_OVERRIDE=$R/build_variants/libfenv_r4base.so timeout -k 10 120 python -u tools/ppo_mb_time.py >> $O/timing.jsonl 2>> $O/timing.err || exit $?
done
cat $O/timing.jsonl
for v in prof1 prof2; do
  FENV_LIB_OVERRIDE=$R/build_variants/libfenv_$v.so timeout -k 10 120 python -u tools/ppo_phase_profile.py > $O/phase_$v.txt 2>&1 || exit $?
done
cat $O/phase_prof1.txt $O/phase_prof2.txt | grep -v amdgpu
bash tools/policy_pmc.sh > $O/policy_pmc.log 2>&1 || { tail -5 $O/policy_pmc.log; exit 1; }
python3 tools/policy_pmc_summary.py gpurun_out $O/r4_policy_pmc_sq.json > /dev/null || exit $?
head -c 1500 $O/r4_policy_pmc_sq.json; echo
FENV_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 \
  --formations 262144 > $O/rehearse_2rank.json 2> $O/rehearse_2rank.err
rc=$?; echo "2-rank rc=$rc"; cut -c1-800 $O/rehearse_2rank.json; tail -3 $O/rehearse_2rank.err
exit $rc
