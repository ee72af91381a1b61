#!/bin/bash
# round 5, first evidence call: shard-size sweep + gloo rehearsal, the MT19937 config-3 test, then
# (last: it is expected to end in the profiler's exit-time SIGSEGV) the cooperative-launch exit
# probe under rocprofv3 with the process's maps dumped for symbolization.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5
mkdir -p $O
tools/scale_rehearsal.sh || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 200 --timeout-method thread \
  -k "mt19937_config3" > $O/pytest_mt3.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_mt3.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/coop_exit" -o p \
  -- python3 "$R/tools/coop_exit_probe.py" "$R/$O/coop_exit" > "$R/$O/coop_exit.out" 2> "$R/$O/coop_exit.err"
echo "coop probe rc=$?"
exit 0
