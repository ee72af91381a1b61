"""Two PPO updates at the reference's training config (seed 0), then the flat parameters, Adam
moments and the loss statistics to an .npz: two library builds that should compute the same
arithmetic are compared bit for bit with `python tools/ppo_params_dump.py --cmp a.npz b.npz`.

    FENV_LIB_OVERRIDE=... python tools/ppo_params_dump.py out.npz
"""
import os
import sys

import numpy as np

if sys.argv[1] == "--cmp":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    for k in a.files:
        same = np.array_equal(a[k].view(np.uint8), b[k].view(np.uint8))
        d = float(np.max(np.abs(a[k].astype(np.float64) - b[k].astype(np.float64))))
        print(f"{k:10s} bit-identical={same} max|diff|={d:.3e}")
    sys.exit(0)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pkgload  # noqa: E402

pkg = pkgload.load()
from importlib import import_module  # noqa: E402

venv = import_module(pkg.__name__ + ".vectorized_env")
ppo_mod = import_module(pkg.__name__ + ".ppo")
dev = torch.device("cuda", 0)
env = venv.FormationEnv({"num_formation": 1000, "num_agents_per_formation": 5, "goal_in_obs": True},
                        device=dev, seed=0, reset_mode="philox")
m = ppo_mod.PPO(env, ppo_mod.PPOConfig(), seed=0)
stats = []
for _ in range(2):
    with torch.no_grad():
        m.collector.collect()
    s = m.train()
    stats.append([float(s[k]) for k in sorted(s) if isinstance(s[k], (int, float))])
torch.cuda.synchronize()
sd = m.opt.state_dict()["state"].get(0, {})
out = {"params": m.param.detach().cpu().numpy(), "stats": np.array(stats, dtype=np.float64)}
for k in ("exp_avg", "exp_avg_sq"):
    if k in sd:
        out[k] = sd[k].cpu().numpy()
np.savez(sys.argv[1], **out)
print("saved", sys.argv[1], stats)
