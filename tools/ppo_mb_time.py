"""us per minibatch of the fused PPO update at the reference's training config (bench.py's
ppo_update_bench; the library FENV_LIB_OVERRIDE names, else the in-tree one).  One JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
import pkgload  # noqa: E402

pkg = pkgload.load()
r = bench.ppo_update_bench(pkg.__name__, torch.device("cuda", 0), updates=3)
r["lib"] = os.path.basename(os.environ.get("FENV_LIB_OVERRIDE", "in-tree"))
print(json.dumps({k: r[k] for k in ("lib", "us_per_minibatch", "ms_per_update")}), flush=True)
