#!/bin/bash
# Interleaved A/B of bench.py argument sets on the driver's window (--steps 20 --warmup 5, secondary
# lines off): for each round, size and variant one bench process; then one summary row per
# variant and size (value, fixed overhead, kernel_value).  Parameters (env):
#   VARIANTS  ';'-separated variants, each bench arguments and/or VAR=value environment settings,
#             e.g. "--issue gated;--issue host" or "ROC_ACTIVE_WAIT_TIMEOUT=2000;--issue gated"
#   SIZES     formations per run (default "131072 1048576"); ROUNDS (default 3); TAG (output dir)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-ab}
mkdir -p "$O"
IFS=';' read -ra V <<< "${VARIANTS:?set VARIANTS}"
for r in $(seq 1 ${ROUNDS:-3}); do
  for F in ${SIZES:-131072 1048576}; do
    for i in "${!V[@]}"; do
      E=(); A=()
      for t in ${V[$i]}; do
        t=${t//RANDOMPORT/$((20000 + RANDOM % 20000))}  # a fresh rendezvous port per process
        case "$t" in --*) A+=("$t");; *=*) E+=("$t");; *) A+=("$t");; esac
      done
      timeout -k 10 120 env "${E[@]}" python bench.py --gpus 1 --steps 20 --warmup 5 --formations $F \
        --no-policy --no-configs --no-cpu-baseline "${A[@]}" > "$O/v${i}_${F}_$r.json" 2> "$O/v${i}_${F}_$r.err" \
        || { echo "FAIL variant $i size $F rc=$?"; tail -3 "$O/v${i}_${F}_$r.err"; exit 1; }
    done
  done
  echo "round $r done"
done
python3 - "$O" "${VARIANTS}" <<'PY'
import glob, json, sys
o, names = sys.argv[1], sys.argv[2].split(";")
rows = {}
for f in sorted(glob.glob(o + "/v*_*_*.json")):
    i, F, _ = f.rsplit("/", 1)[1][1:-5].split("_")
    d = json.loads([x for x in open(f) if x.startswith("{")][-1])
    rows.setdefault((int(F), int(i)), []).append(d)
for (F, i), ds in sorted(rows.items()):
    print(f"{F:>8} [{names[i]}] value", " ".join("%.3e" % d["value"] for d in ds),
          "| fixed us", " ".join("%.1f" % (1e3 * d["fixed_overhead_ms"]) for d in ds),
          "| kernel_value", " ".join("%.3e" % d["kernel_value"] for d in ds))
PY
