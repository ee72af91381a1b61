"""Summarise tools/xlat_pmc.sh: per footprint shape, the unprofiled timing and every PMC counter
averaged over the rollout dispatches, also per 2 MiB of algorithmic bytes (so shapes with
different launch lengths compare directly).  Usage: python tools/xlat_summary.py gpurun_out/xlat"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

out = sys.argv[1]
A, F = 5 * (1 << 20), 1 << 20
STEPS = {"t10": 10.0, "t4same": 4.0, "t4of10": 10.0 / 3.0, "t10alt": 10.0}
res = {}
for case, T in STEPS.items():
    tf = os.path.join(out, f"{case}_time.json")
    if not os.path.exists(tf):
        continue
    r = {"time": json.loads(open(tf).read().strip().splitlines()[-1])}
    bytes_per_dispatch = A * (45 * T + 16) + F * 20
    counters = defaultdict(list)
    for d in sorted(glob.glob(os.path.join(out, f"{case}_*"))):
        if not os.path.isdir(d):
            continue
        for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                if "k_rollout" in row.get("Kernel_Name", ""):
                    counters[row["Counter_Name"]].append(float(row["Counter_Value"]))
    r["per_dispatch"] = {k: sum(v) / len(v) for k, v in sorted(counters.items())}
    r["per_2MiB"] = {k: v / (bytes_per_dispatch / 2 ** 21) for k, v in r["per_dispatch"].items()}
    r["dispatches"] = {k: len(v) for k, v in sorted(counters.items())}
    res[case] = r
print(json.dumps(res, indent=1))
