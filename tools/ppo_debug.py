"""Per-parameter-group difference between the fused ppo_update kernel and the eager torch update
(one epoch over F formations, batch B): prints max |fused - eager| / max |eager - init| per group."""
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


def groups(D):
    H = 64
    names = [("pi0W", H * D), ("pi0b", H), ("pi2W", H * H), ("pi2b", H), ("vf0W", H * D),
             ("vf0b", H), ("vf2W", H * H), ("vf2b", H), ("actW", 2 * H), ("actb", 2),
             ("valW", H), ("valb", 1), ("logstd", 2)]
    o = 0
    for n, k in names:
        yield n, o, o + k
        o += k


for F, bs, ep in ((1, 50, 1), (32, 64, 1), (16, 64, 2)):
    res = []
    for fused in (False, True):
        env = venv.FormationEnv({"num_formation": F, "num_agents_per_formation": 5,
                                 "goal_in_obs": True}, device=DEV, seed=1, reset_mode="philox")
        ppo = ppo_mod.PPO(env, ppo_mod.PPOConfig(batch_size=bs, n_epochs=ep), seed=4,
                          use_graph=False, use_fused=fused)
        f0 = ppo.policy.flat.clone()
        with torch.no_grad():
            ppo.collector.collect()
        st = ppo.train()
        res.append((f0, ppo.policy.flat.clone(), st))
    (a0, p0, s0), (a1, p1, s1) = res
    print(f"F={F} batch={bs} epochs={ep}: stats eager {s0} fused {s1}")
    for n, lo, hi in groups(8):
        mv = (p0[lo:hi] - a0[lo:hi]).abs().max().item()
        er = (p1[lo:hi] - p0[lo:hi]).abs().max().item()
        print(f"  {n:7s} moved {mv:.3e} err {er:.3e} ratio {er / max(mv, 1e-30):.3e}")
