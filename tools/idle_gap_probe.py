"""Why is the first launch after a synchronize slower?  Fused 10-step rollouts at config 3; after
a warm stream of launches, synchronize, idle the host for G ms, then time 3 launches with HIP
events (first, second, third).  G = none (no synchronize: back-to-back), 0, 1, 10, 100 ms."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pkgload  # noqa: E402

pkg = pkgload.load()
from importlib import import_module  # noqa: E402

venv = import_module(pkg.__name__ + ".vectorized_env")
dev = torch.device("cuda", 0)
F, N, T = 1 << 20, 5, 10
env = venv.FormationEnv({"num_formation": F, "num_agents_per_formation": N, "goal_in_obs": True},
                        log=False, device=dev, seed=0, reset_mode="philox")
A = env.num_envs
acts = torch.rand((T, A, 2), device=dev) * 2 - 1
obs = torch.empty((T, A, 8), device=dev)
rew = torch.empty((T, A), device=dev)
done = torch.empty((T, A), dtype=torch.bool, device=dev)
env.reset_tensor()
res = {}
for rep in range(4):
    for gap in (None, 0.0, 1.0, 10.0, 100.0):
        for _ in range(40):
            env.rollout(acts, obs, rew, done)
        if gap is not None:
            torch.cuda.synchronize()
            if gap > 0:
                time.sleep(gap * 1e-3)
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        evs[0].record()
        for k in range(3):
            env.rollout(acts, obs, rew, done)
            evs[k + 1].record()
        torch.cuda.synchronize()
        res.setdefault(gap, []).append([evs[k].elapsed_time(evs[k + 1]) * 1e3 for k in range(3)])
for gap, v in res.items():
    name = "no sync" if gap is None else f"sync + {gap:g} ms"
    print(f"{name:16s} " + "  ".join("[" + ", ".join(f"{x:6.1f}" for x in r) + "]" for r in v), flush=True)
