#!/bin/bash
# Round 4: the driver's bench command with the MT19937-mode secondary line.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4x; mkdir -p "$O"; cd "$R"
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_driver.json" 2> "$O/bench_driver.err"
rc=$?; python3 -c "
import json; d=json.loads([l for l in open('$O/bench_driver.json') if l.startswith('{')][-1])
print(d['value'], d['roofline']['frac']); print(json.dumps(d.get('mt19937_mode')))"; exit $rc
