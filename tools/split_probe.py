"""Does a smaller footprint PER LAUNCH speed up the real env kernel?  Config 3's 1,048,576 x 5
formations as (a) one env and one 10-step launch per step window, or (b) S envs of 1M / S
formations, each with its own buffers, launched back to back (the same total bytes and total
footprint, a 1/S footprint per launch).  HIP events around 20 windows, 3 interleaved rounds.
tools/plane_order_ubench.hip measured +1.5-3 % for S = 2-4 on the bare byte mix."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pkgload  # noqa: E402

pkg = pkgload.load()
from importlib import import_module  # noqa: E402

venv = import_module(pkg.__name__ + ".vectorized_env")
dev = torch.device("cuda", 0)
F, N, T, W = 1 << 20, 5, 10, 20


def setup(S):
    parts = []
    for k in range(S):
        f = F // S
        env = venv.FormationEnv({"num_formation": f, "num_agents_per_formation": N,
                                 "goal_in_obs": True}, log=False, device=dev, seed=k,
                                reset_mode="philox", first_formation=k * f, total_formations=F)
        A = env.num_envs
        bufs = (torch.rand((T, A, 2), device=dev) * 2 - 1, torch.empty((T, A, 8), device=dev),
                torch.empty((T, A), device=dev), torch.empty((T, A), dtype=torch.bool, device=dev))
        env.reset_tensor()
        parts.append((env, bufs))
    return parts


def window(parts):
    for env, (a, o, r, d) in parts:
        env.rollout(a, o, r, d)


res = {}
setups = {S: setup(S) for S in (1, 2, 4)}
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for rnd in range(3):
    for S, parts in setups.items():
        for _ in range(5):
            window(parts)
        e0.record()
        for _ in range(W):
            window(parts)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / W
        res.setdefault(S, []).append(ms)
for S, v in res.items():
    print(json.dumps({"S": S, "ms_per_10_steps": v, "agent_steps_per_s": [F * N * T / (m * 1e-3) for m in v]}))
