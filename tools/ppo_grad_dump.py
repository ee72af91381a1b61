"""Diagnostic (needs build_variants/libfenv_dump.so, -DFENV_PPO_DUMP_GRAD=1): the fused kernel's
raw gradient of a single 50-sample minibatch vs the eager torch gradient, W1 blocks per column."""
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
out = []
for fused in (False, True):
    env = venv.FormationEnv({"num_formation": 1, "num_agents_per_formation": 5,
                             "goal_in_obs": True}, device=DEV, seed=1, reset_mode="philox")
    ppo = ppo_mod.PPO(env, ppo_mod.PPOConfig(batch_size=50, n_epochs=1), seed=4,
                      use_graph=False, use_fused=fused)
    with torch.no_grad():
        ppo.collector.collect()
    if fused:
        ppo.train()
        out.append(ppo.opt.state[ppo.param]["exp_avg"].clone())
        obs = ppo._flat()[0]
    else:
        ppo._forward_backward(torch.arange(50, device=DEV))
        out.append(ppo.param.grad.clone())
e, f = out
torch.set_printoptions(precision=4, linewidth=200, sci_mode=True)
for name, lo in (("pi0W", 0), ("vf0W", 4736)):
    E = e[lo:lo + 512].view(64, 8)
    Fm = f[lo:lo + 512].view(64, 8)
    print(name, "per-column max|fused-eager| / max|eager|:")
    print(((Fm - E).abs().amax(0) / E.abs().amax(0)).cpu())
    print("rows 0-2 eager", E[:3].cpu(), "\nrows 0-2 fused", Fm[:3].cpu())
print("other groups max rel err", ((f[512:4736] - e[512:4736]).abs().max() / e[512:4736].abs().max()).item(),
      ((f[5248:] - e[5248:]).abs().max() / e[5248:].abs().max()).item())
print("obs column means", obs.mean(0).cpu(), "abs max", obs.abs().amax(0).cpu())
# internal consistency of the dump: O rows vs the buffer's observations, GW1 vs dZ1^T . O
sq = ppo.opt.state[ppo.param]["exp_avg_sq"]
O = sq[:576].view(64, 9)[:50, :8]
Z = sq[576:576 + 8192].view(2, 64, 64)[:, :50]
obs_s = obs[torch.argsort(obs[:, 0] * 1000 + obs[:, 1])]
O_s = O[torch.argsort(O[:, 0] * 1000 + O[:, 1])]
print("O rows == obs rows (as sets):", torch.equal(O_s, obs_s), (O_s - obs_s).abs().max().item())
for net, lo in ((0, 0), (1, 4736)):
    gw1 = Z[net].T @ O
    print(f"net {net}: |GW1_dump - dZ1^T O| / |GW1| =",
          ((f[lo:lo + 512].view(64, 8) - gw1).abs().max() / gw1.abs().max()).item(),
          " |b1_dump - sum dZ1| =", (f[lo + 512:lo + 576] - Z[net].sum(0)).abs().max().item())
O9 = sq[:576].view(64, 9)
print("O dump rows 0-5 (9 cols):\n", O9[:6].cpu())
print("obs rows 0-5:\n", obs[:6].cpu())
bad = (O9[:50, :8].unsqueeze(1) - obs.unsqueeze(0)).abs().amax(2).amin(1)  # distance to nearest obs row
print("per-row distance to nearest obs row:", bad.cpu())
