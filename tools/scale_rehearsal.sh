#!/bin/bash
# bench.py's timed region at the shard sizes of an 8/4/2/1-GPU strong-scaling run of config 3
# (131072, 262144, 524288, 1048576 formations on one GPU, the driver's --steps 20 --warmup 5):
# the fixed overhead (wall - event-timed kernel span) of the gated window and of the host-issued
# window nested in the same line, per size; then the bench's N > 1 path
# with two ranks on the one GPU over gloo (its rate says nothing about scaling).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r5}
O=gpurun_out/$TAG
mkdir -p "$O"
export PYTHONUNBUFFERED=1
for F in ${SIZES:-131072 262144 524288 1048576}; do
  for rep in $(seq 1 ${REPS:-3}); do
    timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --formations $F --no-policy \
      --no-configs --no-cpu-baseline > "$O/shard_${F}_$rep.json" 2> "$O/shard_${F}_$rep.err" || exit $?
  done
done
python - "$O" <<'PY'
import glob, json, sys
rows = {}
for f in sorted(glob.glob(sys.argv[1] + "/shard_*_*.json")):
    d = json.load(open(f))
    F = d["config"]["formations"]
    h = d.get("host_issued", d)
    rows.setdefault(F, []).append((d.get("issue", "host"), d["fixed_overhead_ms"] * 1e3,
                                   h["fixed_overhead_ms"] * 1e3, d["value"], h["value"],
                                   d["kernel_value"]))
for F, v in sorted(rows.items()):
    print(F, "fixed us (%s):" % v[0][0], " ".join("%.1f" % r[1] for r in v),
          "| host-issued fixed us:", " ".join("%.1f" % r[2] for r in v))
    print(F, "value:", " ".join("%.3e" % r[3] for r in v), "| host-issued value:",
          " ".join("%.3e" % r[4] for r in v), "| kernel_value:", " ".join("%.3e" % r[5] for r in v))
PY
if [ -z "${SKIP_GLOO:-}" ]; then
  FENV_DIST_BACKEND=gloo timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 \
    --formations 262144 > "$O/rehearse_2rank.json" 2> "$O/rehearse_2rank.err"
  rc=$?; echo "2-rank rc=$rc"; cut -c1-400 "$O/rehearse_2rank.json"; exit $rc
fi
