"""One bench.ppo_update_bench run (the fused PPO update at the reference's training config) for
tools/ppo_pmc.sh's rocprofv3 --pmc passes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.argv = ["x"]
import torch  # noqa: E402

import bench  # noqa: E402
import pkgload  # noqa: E402

pkg = pkgload.load()
print(bench.ppo_update_bench(pkg.__name__, torch.device("cuda", 0)), flush=True)
