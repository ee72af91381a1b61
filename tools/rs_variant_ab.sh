#!/bin/bash
# Same-box A/B of k_rollout_wave_rs builds (build_variants/libfenv_<tag>.so vs the in-tree
# libfenv.so): a parity subset on each variant first (staged-kernel sizes vs the C oracle, NULL
# outputs, config-3 sampled), then interleaved timing rounds of tools/xlat_probe.py (t10 = the
# bench's shape, t4same) and the driver's bench command.  VARIANTS="ob obxpf" ROUNDS=2.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out/rsab"
mkdir -p "$O"
VARIANTS=${VARIANTS:-"ob obxpf xpf"}
ROUNDS=${ROUNDS:-2}
export PYTHONUNBUFFERED=1
libs="base"
for v in $VARIANTS; do libs="$libs $v"; done
libpath() { if [ "$1" = base ]; then echo "$R/marl-distributedformation_amd/libfenv.so"; else echo "$R/build_variants/libfenv_$1.so"; fi; }
if [ -z "${SKIP_PARITY:-}" ]; then
  for v in $VARIANTS; do
    FENV_LIB_OVERRIDE=$(libpath $v) timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
      tests/test_gpu_parity.py tests/test_gpu_fullsize.py \
      -k "staged_kernel or null_outputs or stats_records or extreme or full_size_sampled" > "$O/parity_$v.log" 2>&1
    rc=$?; echo "parity $v rc=$rc: $(tail -1 "$O/parity_$v.log")"
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  done
fi
for r in $(seq 1 "$ROUNDS"); do
  for v in $libs; do
    L=$(libpath $v)
    for c in t10 t4same; do
      out=$(FENV_LIB_OVERRIDE=$L timeout -k 10 120 python tools/xlat_probe.py $c --launches 40) || { echo "probe $v $c failed"; exit 1; }
      echo "round $r $v $out"
    done
    out=$(FENV_LIB_OVERRIDE=$L timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-policy --no-configs 2>/dev/null) || { echo "bench $v failed"; exit 1; }
    echo "round $r $v bench $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("ms_per_step", d["ms_per_step"], "frac", d["roofline"]["frac"])')"
  done
done
