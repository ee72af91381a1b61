"""The fused policy rollout at BASELINE config 2 (65,536 x 10, bench.py's policy_rollout_bench):
kernel ms per 10-step rollout, for the library FENV_LIB_OVERRIDE names (else the in-tree one).
One JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
import pkgload  # noqa: E402

pkg = pkgload.load()
r = bench.policy_rollout_bench(pkg.__name__, torch.device("cuda", 0), 65536, 10, 10)
print(json.dumps({"lib": os.path.basename(os.environ.get("FENV_LIB_OVERRIDE", "in-tree")),
                  "rollout_kernel_ms": r["rollout_kernel_ms"], "value": r["value"],
                  "valu_frac": r["roofline"]["frac"]}), flush=True)
