"""Which MT19937-mode rollout calls block the host, and for how long: config 3 (1,048,576 x 5),
10-step calls over 3,010 steps (reset events at steps 1,001, 2,003, 3,005 after env.reset), every
call's host time over 1 ms listed with its step.  The GPU queue is bounded by a synchronize every
`sync_every` calls (0: never), so the run also shows whether a blocked call starves the GPU.
    python tools/mt_host_block_probe.py [sync_every]   -> one JSON line
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
F, N, T, STEPS = 1 << 20, 5, 10, 3010
SYNC = int(sys.argv[1]) if len(sys.argv) > 1 else 0
t_create = time.perf_counter()
env = ve.FormationEnv({"num_formation": F, "num_agents_per_formation": N, "goal_in_obs": True},
                      log=False, device=DEV, seed=0, reset_mode="mt19937")
t_create = time.perf_counter() - t_create
A = env.num_envs
acts = torch.rand((T, A, 2), device=DEV) * 2 - 1
obs = torch.empty((T, A, 8), device=DEV)
rew = torch.empty((T, A), device=DEV)
done = torch.empty((T, A), dtype=torch.bool, device=DEV)
t_reset = time.perf_counter()
env.reset_tensor()
t_reset = time.perf_counter() - t_reset
torch.cuda.synchronize()
slow = []
k = 0
t0 = time.perf_counter()
n = 0
while k < STEPS:
    L = min(T, STEPS - k)
    t1 = time.perf_counter()
    env.rollout(acts[:L], obs[:L], rew[:L], done[:L])
    dt = time.perf_counter() - t1
    if dt > 1e-3:
        slow.append({"step": k, "host_ms": round(1e3 * dt, 2)})
    k += L
    n += 1
    if SYNC and n % SYNC == 0:
        torch.cuda.synchronize()
torch.cuda.synchronize()
el = time.perf_counter() - t0
print(json.dumps({"create_ms": round(1e3 * t_create, 1), "reset_ms": round(1e3 * t_reset, 1),
                  "sync_every": SYNC, "agent_steps_per_s": A * STEPS / el, "slow_calls": slow}),
      flush=True)
env.release()
