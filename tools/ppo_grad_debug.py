"""One-minibatch gradient check of the fused ppo_update kernel: after one Adam step exp_avg =
(1 - beta1) * clip_coef * grad, so the normalised exp_avg of the fused and eager updates must
agree; prints the per-group relative error of the normalised gradients."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pkgload  # noqa: E402
from importlib import import_module  # noqa: E402

pkg = pkgload.load()
venv = import_module(pkg.__name__ + ".vectorized_env")
ppo_mod = import_module(pkg.__name__ + ".ppo")
DEV = torch.device("cuda", 0)
H = 64
names = [("pi0W", H * 8), ("pi0b", H), ("pi2W", H * H), ("pi2b", H), ("vf0W", H * 8),
         ("vf0b", H), ("vf2W", H * H), ("vf2b", H), ("actW", 2 * H), ("actb", 2),
         ("valW", H), ("valb", 1), ("logstd", 2)]
for F, bs in ((1, 50), (2, 64)):
    g = []
    for fused in (False, True):
        env = venv.FormationEnv({"num_formation": F, "num_agents_per_formation": 5,
                                 "goal_in_obs": True}, device=DEV, seed=1, reset_mode="philox")
        ppo = ppo_mod.PPO(env, ppo_mod.PPOConfig(batch_size=bs, n_epochs=1), seed=4,
                          use_graph=False, use_fused=fused)
        with torch.no_grad():
            ppo.collector.collect()
        ppo.train()
        m = ppo.opt.state[ppo.param]["exp_avg"].clone()
        g.append(m / m.norm())
    print(f"F={F} batch={bs} (first minibatch of {F * 50} samples)")
    o = 0
    for n, k in names:
        a, b = g[0][o:o + k], g[1][o:o + k]
        print(f"  {n:7s} |g| {a.norm().item():.3e} rel err {((b - a).norm() / a.norm()).item():.3e}"
              f"  fused/eager norm {(b.norm() / a.norm()).item():.4f}")
        o += k
