#!/bin/bash
# round 5: the policy kernels' 1 + 2^y adds as v_pk_add_f32 (pk1, in-tree) vs one v_add_f32 each
# (pk0): the policy / rollout parity tests on the in-tree library, then 3 interleaved rounds of the
# fused policy rollout at config 2 (tools/policy_rollout_time.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5m
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_policy.py tests/test_gpu_rollout.py tests/test_gpu_fullsize.py -x -v \
  --timeout 200 --timeout-method thread -k "policy or rollout" > $O/pytest_policy.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_policy.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in pk0 pk1; do
    FENV_LIB_OVERRIDE=build_variants/libfenv_$v.so timeout -k 10 120 python tools/policy_rollout_time.py \
      > $O/${v}_$r.json 2> $O/${v}_$r.err || exit $?
    echo "$v $r: $(cat $O/${v}_$r.json)"
  done
done
