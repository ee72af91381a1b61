#!/bin/bash
# Round 4: the config-3 Philox kernel forced to 8 waves/SIMD (amdgpu_waves_per_eu(8): 64 VGPRs, no spill,
# 4 workgroups/CU instead of 3; build_variants/libfenv_occ8.so) vs in-tree: the driver bench command, x2.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4u; mkdir -p "$O"; cd "$R"
for k in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$O/intree_$k.json" 2>> "$O/err.txt" || exit 1
  FENV_LIB_OVERRIDE=$R/build_variants/libfenv_occ8.so timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline \
    > "$O/occ8_$k.json" 2>> "$O/err.txt" || exit 1
done
python3 - "$O" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    r = d["roofline"]; ra = d.get("random_action_rollout", {})
    print(os.path.basename(f), round(d["value"] / 1e9, 2), "frac", round(r["frac"], 4), "kernel_ms", round(r["avg_kernel_ms"], 4),
          "ceil", round(r["same_box_ceiling"]["kernel_frac_of_ceiling"], 3), "random_ms", ra.get("avg_kernel_ms"),
          "single", d.get("single_step", {}).get("avg_kernel_ms"), "cfg1", d.get("env_configs", {}).get("config1", {}).get("avg_kernel_ms"),
          "cfg4", d.get("env_configs", {}).get("config4", {}).get("avg_kernel_ms"))
PY
