"""Summarise rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) for the rollout kernel into
profiles/pmc_traffic.json.  gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports
half the bytes of a wide coalesced streaming read, so read bytes = 2 x FETCH_SIZE (KiB);
WRITE_SIZE is exact for 16-B-per-lane streaming stores."""
import csv
import glob
import json
import os
import sys

out_dir, tag = sys.argv[1], sys.argv[2]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_dispatch(counter):
    files = glob.glob(os.path.join(out_dir, f"pmc_{tag}_{counter}", "**", "*counter_collection*.csv"),
                      recursive=True)
    vals = []
    for f in files:
        for row in csv.DictReader(open(f)):
            if "k_rollout_wave" in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                vals.append(float(row["Counter_Value"]))
    return vals


fetch = per_dispatch("FETCH_SIZE")
write = per_dispatch("WRITE_SIZE")
if not fetch or not write:
    print("no rollout dispatches found", file=sys.stderr)
    sys.exit(1)
f_kb = sum(fetch) / len(fetch)
w_kb = sum(write) / len(write)
res = {
    "workload": "config3: 1048576 formations x 5 agents (1048576 per GPU x 1), fused 10-step rollouts, philox resets",
    "kernel": "k_rollout_wave_rs",
    "dispatches": [len(fetch), len(write)],
    "FETCH_SIZE_kib_per_launch": f_kb,
    "WRITE_SIZE_kib_per_launch": w_kb,
    "read_bytes_per_launch_corrected": 2 * f_kb * 1024,
    "write_bytes_per_launch": w_kb * 1024,
    "hbm_bytes_per_launch": (2 * f_kb + w_kb) * 1024,
    "note": "read side doubled per the gfx950 FETCH_SIZE calibration (wide streaming reads)",
}
os.makedirs(os.path.join(root, "profiles"), exist_ok=True)
json.dump(res, open(os.path.join(out_dir, f"pmc_traffic_{tag}.json"), "w"), indent=1)
print(json.dumps(res, indent=1))
