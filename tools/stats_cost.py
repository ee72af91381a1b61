"""In-kernel cost of the per-4-wave {reward, done} stats records at the headline size: fused
10-step rollouts alternating partial=records / partial=None in one process (HIP events around
each launch on the launch stream), so box and clock drift cancel.  Library: in-tree or
FENV_LIB_OVERRIDE."""
import os
import sys

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
part = torch.zeros((env.partial_count(), 2), device=dev)
env.reset_tensor()
for _ in range(100):
    env.rollout(acts, obs, rew, done, partial=part)
torch.cuda.synchronize()
K = int(os.environ.get("LAUNCHES", "400"))
evs = [torch.cuda.Event(enable_timing=True) for _ in range(K + 1)]
evs[0].record()
for k in range(K):
    env.rollout(acts, obs, rew, done, partial=part if k % 2 == 0 else None)
    evs[k + 1].record()
torch.cuda.synchronize()
ms = [evs[k].elapsed_time(evs[k + 1]) for k in range(K)]
with_s = sorted(ms[0::2])
without = sorted(ms[1::2])
med = lambda v: v[len(v) // 2]  # noqa: E731
lib = os.path.basename(os.environ.get("FENV_LIB_OVERRIDE", "in-tree"))
print(f"{lib:24s} stats {med(with_s) * 1e3:7.1f} us (mean {sum(with_s) / len(with_s) * 1e3:7.1f})  "
      f"no stats {med(without) * 1e3:7.1f} us (mean {sum(without) / len(without) * 1e3:7.1f})  "
      f"diff of medians {(med(with_s) - med(without)) * 1e3:+.1f} us", flush=True)
