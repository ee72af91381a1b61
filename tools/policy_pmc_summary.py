"""Average the rocprofv3 SQ/GRBM PMC passes of tools/policy_pmc.sh per kernel and per dispatch
-> JSON (profiles/<tag>_policy_pmc_sq.json).  Units as rocprofv3 reports them: SQ_*_CYCLES,
SQ_ACTIVE_INST_* and SQ_WAIT_* count quad-cycles, SQ_VALU_MFMA_BUSY_CYCLES cycles
(MI355X_MICROARCH.md, PMC units row); all summed over the chip.

    python tools/policy_pmc_summary.py gpurun_out profiles/r2_policy_pmc_sq.json"""
import collections
import csv
import glob
import json
import os
import sys

src, out = sys.argv[1], sys.argv[2]
kpat = sys.argv[3] if len(sys.argv) > 3 else "k_policy"  # kernel-name filter
prefix = sys.argv[4] if len(sys.argv) > 4 else "ppmc_"   # output directories of the passes
what = sys.argv[5] if len(sys.argv) > 5 else ("tools/policy_pmc.sh) over tools/rollout_timing.py, "
                                               "config 2 (65536 x 10)")
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(src, prefix + "*", "**", "*counter_collection*.csv"), recursive=True):
    per = collections.defaultdict(float)  # (kernel, dispatch, counter) -> value (sum over dims)
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "")
        if kpat not in k:
            continue
        per[(k.split("(")[0], row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
    for (k, _, c), v in per.items():
        acc[k][c].append(v)
res = {"source": "rocprofv3 --pmc passes (" + what + ", per dispatch averages",
       "units": "SQ_* cycle counters in quad-cycles except SQ_VALU_MFMA_BUSY_CYCLES; summed over "
                "the chip",
       "kernels": {k: {c: sum(v) / len(v) for c, v in sorted(cs.items())}
                   for k, cs in sorted(acc.items())},
       "dispatches": {k: {c: len(v) for c, v in sorted(cs.items())} for k, cs in sorted(acc.items())}}
os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res["kernels"], indent=1))
