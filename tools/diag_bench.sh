set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/diag
B="python bench.py --no-policy --no-configs --no-cpu-baseline"
for a in "--steps 20 --warmup 5" "--steps 20 --warmup 5 --episode-phase aligned" "--steps 200 --warmup 5" "--steps 20 --warmup 5 --no-stats"; do
  timeout -k 10 120 $B $a > gpurun_out/diag/out.json 2>gpurun_out/diag/err.txt || { echo "rc=$?"; cat gpurun_out/diag/err.txt; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/diag/out.json'));r=d['roofline'];print('$a', 'ms/step',round(d['ms_per_step'],4),'avg',round(r['avg_kernel_ms'],4),'min',round(r['launch_ms_min'],4),'max',round(r['launch_ms_max'],4),'frac',round(r['frac'],3),'issue_ms',round(d['host_issue_ms'],3),'pw',d['warmup_launches'],round(d['warmup_ms'],1))"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/diag/prof" -o b -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --no-policy --no-configs --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/diag/prof.json" 2>&1
echo "prof rc=$?"
