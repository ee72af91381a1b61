"""Stress of the two-CU fused PPO update's gradient-norm exchange: K updates at the reference's
training config in one process (FENV_LIB_OVERRIDE picks the library), each timed; counts the
updates that ended in NaN (raised by ppo.py) and the launches ppo.py re-ran after a lost
exchange.  A lost exchange costs the spin budget (seconds), so its updates stand out in time."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pkgload  # noqa: E402

pkg = pkgload.load()
from importlib import import_module  # noqa: E402

venv = import_module(pkg.__name__ + ".vectorized_env")
ppo_mod = import_module(pkg.__name__ + ".ppo")
dev = torch.device("cuda", 0)
K = int(os.environ.get("K", "100"))
env = venv.FormationEnv({"num_formation": 1000, "num_agents_per_formation": 5, "goal_in_obs": True},
                        log=False, device=dev, seed=0, reset_mode="philox")


def fresh(seed):
    return ppo_mod.PPO(env, ppo_mod.PPOConfig(), seed=seed)


m = fresh(0)
fails, slow, times = 0, 0, []
for k in range(K):
    with torch.no_grad():
        m.collector.collect()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    try:
        m.train()
        ok = True
    except RuntimeError as e:
        ok = False
        fails += 1
        print(f"update {k}: {e}", flush=True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) * 1e3
    times.append(dt)
    if dt > 500:
        slow += 1
        print(f"update {k}: {dt:.0f} ms", flush=True)
    if not ok:
        m = fresh(k + 1)
    if k % 20 == 0:
        print(f"{k} updates, {fails} failed, {getattr(m, 'exchange_retries', 0)} re-runs "
              f"(current model), median {sorted(times)[len(times) // 2]:.1f} ms", flush=True)
print(f"{os.path.basename(os.environ.get('FENV_LIB_OVERRIDE', 'in-tree'))}: {K} updates, "
      f"{fails} failed, {slow} over 500 ms, median {sorted(times)[len(times) // 2]:.1f} ms, "
      f"re-runs (last model) {getattr(m, 'exchange_retries', 0)}", flush=True)
