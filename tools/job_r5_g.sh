#!/bin/bash
# round 5: the rollout byte mix's HBM rate against the launch footprint (tools/plane_order_ubench,
# slice order, T = 10, SPLIT_ONLY rows: slice + split variants) for A = 1M ... 8M agents
# (0.47 ... 3.8 GB per launch).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5o
mkdir -p $O
for A in 1048576 2097152 3145728 4194304 5242880 6291456 8388608; do
  SPLIT_ONLY=1 timeout -k 10 60 tools/plane_order_ubench $A 10 > $O/fp_$A.jsonl 2>&1 || exit $?
  python3 -c "
import json
rows=[json.loads(l) for l in open('$O/fp_$A.jsonl')]
s=[r for r in rows if r['order']=='slice']
print($A, round(45*$A*10/1e9,2), 'GB', ' '.join('nt%d %.3f' % (r['nt'], r['tb_s']) for r in s))"
done
