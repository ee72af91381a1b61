"""Kernel-only durations of config 1 (4,096 x 5) rollouts for rocprofv3 --kernel-trace --stats:
T=10 (prefetch-4 / split kernel) and T=2 (prefetch-1) launches, 2,000 each, all outputs."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pkgload  # noqa: E402

pkg = pkgload.load()
from importlib import import_module  # noqa: E402

venv = import_module(pkg.__name__ + ".vectorized_env")
dev = torch.device("cuda", 0)
F, N = int(os.environ.get("F", 4096)), int(os.environ.get("N", 5))
env = venv.FormationEnv({"num_formation": F, "num_agents_per_formation": N, "goal_in_obs": True},
                        device=dev, seed=0, reset_mode="philox")
A = env.num_envs
acts = torch.rand((10, A, 2), device=dev) * 2 - 1
obs = torch.empty((10, A, 8), device=dev)
rew = torch.empty((10, A), device=dev)
done = torch.empty((10, A), dtype=torch.bool, device=dev)
for T in (10, 2):
    for _ in range(int(os.environ.get("LAUNCHES", 2000))):
        env.rollout(acts[:T], obs[:T], rew[:T], done[:T])
    torch.cuda.synchronize()
print("done", env.rollout_kernel_name(10), env.rollout_kernel_name(2))
