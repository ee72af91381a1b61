"""One fresh process's FIRST fused PPO update at the reference's training config (as bench.py's
ppo_update line starts): prints its wall time, outcome and ppo.py's re-runs after a lost norm
exchange (a lost exchange spends the spin budget, so it shows in the time)."""
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
env = venv.FormationEnv({"num_formation": 1000, "num_agents_per_formation": 5, "goal_in_obs": True},
                        log=False, device=dev, seed=0, reset_mode="philox")
m = ppo_mod.PPO(env, ppo_mod.PPOConfig(), seed=0)
with torch.no_grad():
    m.collector.collect()
torch.cuda.synchronize()
t0 = time.perf_counter()
try:
    m.train()
    out = "ok"
except RuntimeError as e:
    out = str(e)
torch.cuda.synchronize()
print(f"{sys.argv[1] if len(sys.argv) > 1 else ''} first update {(time.perf_counter() - t0) * 1e3:.0f} ms, "
      f"re-runs {getattr(m, 'exchange_retries', 0)}: {out}", flush=True)
