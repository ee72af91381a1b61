#!/bin/bash
# round 5: does the allocation kind move the footprint knee of the byte mix (slice order, T = 10)?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5p
mkdir -p $O
for al in default contig one; do
  for A in 3145728 5242880; do
    ALLOC=$al SPLIT_ONLY=1 timeout -k 10 60 tools/plane_order_ubench $A 10 > $O/${al}_$A.jsonl 2>&1 || { echo "$al $A rc=$?"; continue; }
    python3 -c "
import json
rows=[json.loads(l) for l in open('$O/${al}_$A.jsonl')]
s=[r for r in rows if r['order']=='slice']
print('$al', $A, round(45*$A*10/1e9,2), 'GB', ' '.join('nt%d %.3f' % (r['nt'], r['tb_s']) for r in s))"
  done
done
