"""Repeat the PPO HIP-graph capture (batch 256) with each BLAS backend preference and count
capture failures (hipBLASLt's bias-fused addmm has been seen to fail inside capture)."""
import os
import sys
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pkgload  # noqa: E402
from importlib import import_module  # noqa: E402

pkg = pkgload.load()
ve = import_module(pkg.__name__ + ".vectorized_env")
ppo_m = import_module(pkg.__name__ + ".ppo")
backend = sys.argv[1] if len(sys.argv) > 1 else "default"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
first = int(sys.argv[3]) if len(sys.argv) > 3 else 0
torch.backends.cuda.preferred_blas_library(backend)
fails = 0
for r in range(first, first + reps):
    env = ve.FormationEnv({"num_formation": 16, "num_agents_per_formation": 5, "goal_in_obs": True},
                          device="cuda:0", seed=r, reset_mode="philox")
    ppo = ppo_m.PPO(env, ppo_m.PPOConfig(batch_size=256, n_epochs=2), seed=r, use_graph=True)
    try:
        with torch.no_grad():
            ppo.collector.collect()
        ppo.train()
        torch.cuda.synchronize()
    except Exception as e:  # noqa: BLE001
        fails += 1
        print(f"rep {r}: {type(e).__name__}: {str(e).splitlines()[0]}", flush=True)
        break
    if os.environ.get("PROBE_GC"):
        del ppo, env
        import gc
        gc.collect()
print(f"{backend}: {fails} failure(s) in {r + 1 - first} captures from seed {first}", flush=True)
