#!/bin/bash
# Same-box A/B of bench.py against bench_head.py (a previous bench.py at the repo root): the
# driver's short command, 3 interleaved rounds, then one default run of bench.py.
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/abi; mkdir -p $O
[ -f bench_head.py ] || git show HEAD~:bench.py > bench_head.py 2>/dev/null || { echo "need bench_head.py (the previous bench.py)"; exit 1; }
for i in 1 2 3; do
  for b in bench_head bench; do
    timeout -k 10 120 python $b.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-policy --no-configs > $O/${b}_$i.json 2>$O/${b}_$i.err || { echo "rc=$? $b"; tail -5 $O/${b}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${b}_$i.json')); r=d['roofline']; print('$b $i frac', round(r['frac'], 4), [round(x, 4) for x in r['launch_ms_first']], 'ms/step', round(d['ms_per_step'], 4), 'issue_ms', round(d['host_issue_ms'],3), 'value %.3e' % d['value'])"
  done
done
timeout -k 10 300 python bench.py > $O/default.json 2>$O/default.err || { echo "default rc=$?"; tail -5 $O/default.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/default.json')); r=d['roofline']; print('default frac', round(r['frac'], 4), 'ms/step', round(d['ms_per_step'], 4), 'value %.3e' % d['value'])"
