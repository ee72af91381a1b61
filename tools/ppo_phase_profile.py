"""Per-phase shader-clock profile of the fused PPO update (diagnostic build with
-DFENV_PPO_PROFILE=1, loaded through FENV_LIB_OVERRIDE): one update at the reference's training
config, cycles per minibatch per phase."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pkgload  # noqa: E402

pkg = pkgload.load()
from importlib import import_module  # noqa: E402

venv = import_module(pkg.__name__ + ".vectorized_env")
ppo_mod = import_module(pkg.__name__ + ".ppo")
_lib = import_module(pkg.__name__ + "._lib")
dev = torch.device("cuda", 0)
env = venv.FormationEnv({"num_formation": 1000, "num_agents_per_formation": 5, "goal_in_obs": True},
                        device=dev, seed=0, reset_mode="philox")
m = ppo_mod.PPO(env, ppo_mod.PPOConfig(), seed=0)
with torch.no_grad():
    m.collector.collect()
m.train()
with torch.no_grad():
    m.collector.collect()
m._sums = torch.zeros(16, dtype=torch.float64, device=dev)
m.train()
torch.cuda.synchronize()
n = env.num_envs * 10
mb = 10 * -(-n // 64)
names = ["gather", "advnorm+layer1", "layer2+heads", "loss", "head grads+dz2", "-", "W2 grads+dh1", "dz1 store",
         "W1 grads", "norm reduce", "adam"]
tot = 0.0
for k, v in zip(names, m._sums[4:15].tolist()):
    print(f"{k:16s} {v / mb:9.0f} cycles/minibatch")
    tot += v / mb
print(f"{'total':16s} {tot:9.0f} cycles/minibatch")
