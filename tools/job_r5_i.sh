#!/bin/bash
# round 5: the footprint knee of the byte mix with and without the action reads (NOACT): is it
# the 256 MB Infinity Cache holding the re-read actions across launches?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5q
mkdir -p $O
for na in 0 1; do
  for A in 2097152 3145728 4194304 5242880; do
    X=""; [ $na = 1 ] && export NOACT=1 || unset NOACT
    SPLIT_ONLY=1 timeout -k 10 60 tools/plane_order_ubench $A 10 > $O/na${na}_$A.jsonl 2>&1 || { echo "rc=$?"; exit 1; }
    python3 -c "
import json
rows=[json.loads(l) for l in open('$O/na${na}_$A.jsonl')]
s=[r for r in rows if r['order']=='slice']
print('noact=$na', $A, 'actions %.2f GB' % (8*$A*10/1e9), ' '.join('nt%d %.3f ms' % (r['nt'], r['ms']) for r in s))"
  done
done
