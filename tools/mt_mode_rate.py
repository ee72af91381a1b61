"""Env rollout rate in MT19937 reset mode (the reference's exact RNG stream) against Philox, at
BASELINE config 3 (1,048,576 x 5) or the size given, over a window that holds reset events
(episode = 1002 steps).  MT19937 mode draws every reset set on the host (std::mt19937 replay of
torch's global stream): what that costs the rollout is the difference between the two lines.

    python tools/mt_mode_rate.py [formations] [steps] [modes]   -> one JSON line per mode
                                                                (modes: philox,mt19937)
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pkgload  # noqa: E402

pkg = pkgload.load()
from importlib import import_module  # noqa: E402

ve = import_module(pkg.__name__ + ".vectorized_env")
DEV = "cuda:0"
F = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
STEPS = int(sys.argv[2]) if len(sys.argv) > 2 else 3010
N, T = 5, 10

MODES = sys.argv[3].split(",") if len(sys.argv) > 3 else ["philox", "mt19937"]
for mode in MODES:
    env = ve.FormationEnv({"num_formation": F, "num_agents_per_formation": N, "goal_in_obs": True},
                          log=False, device=DEV, seed=0, reset_mode=mode)
    A = env.num_envs
    acts = torch.rand((T, A, 2), device=DEV) * 2 - 1
    obs = torch.empty((T, A, 8), device=DEV)
    rew = torch.empty((T, A), device=DEV)
    done = torch.empty((T, A), dtype=torch.bool, device=DEV)
    env.reset_tensor()
    for _ in range(5):
        env.rollout(acts, obs, rew, done)
    torch.cuda.synchronize()
    t_max = 0.0
    t0 = time.perf_counter()
    k = 0
    while k < STEPS:
        L = min(T, STEPS - k)
        t1 = time.perf_counter()
        env.rollout(acts[:L], obs[:L], rew[:L], done[:L])
        dt = time.perf_counter() - t1
        t_max = max(t_max, dt)
        k += L
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(json.dumps({"mode": mode, "formations": F, "steps": STEPS, "agent_steps_per_s": A * STEPS / el,
                      "ms_per_step": 1e3 * el / STEPS, "max_host_ms_per_call": 1e3 * t_max}),
          flush=True)
    env.release()
    del env
    torch.cuda.empty_cache()
