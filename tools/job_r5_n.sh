#!/bin/bash
# round 5: the numpy faces read / write device-mapped host memory in place (fenv_host_alloc):
# the GPU suite at the new library, then the numpy-face probe at configs 0, 2, 3 and 4's shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5n
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest exit $?"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for a in "1000 5 400" "65536 10 100" "1048576 5 20" "16384 64 50"; do
  timeout -k 10 200 python tools/numpy_face_probe.py $a >> $O/probe.jsonl 2>>$O/probe.err || exit 1
done
cat $O/probe.jsonl
