set -u
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for a in torch contig onechunk; do
    for c in t10 t4same; do
      out=$(timeout -k 10 120 python tools/xlat_probe.py $c --alloc $a --launches 40) || { echo "probe $a $c failed"; exit 1; }
      echo "round $r $out"
    done
  done
done
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_ppo_dp.py > gpurun_out/newtests2.log 2>&1; echo "ppo_dp tests rc=$?"; grep -E "PASSED|FAILED|passed|failed|reference-config" gpurun_out/newtests2.log
PAIRS=3 VARIANTS=latepg timeout -k 10 600 bash tools/ppo_variant_ab.sh
