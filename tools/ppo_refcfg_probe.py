"""One PPO update at the reference's training config (1,000 x 5, n_steps 10, batch 64, 10 epochs;
the same seeds as tests/test_gpu_ppo_dp.py::test_fused_update_vs_torch_at_reference_config):
prints the loss means and the final log_std of the fused kernel (the library FENV_LIB_OVERRIDE
names, else the in-tree one) and, with argument 'torch', of the torch graph path, for comparing
kernel variants' numerics without the whole test."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pkgload  # noqa: E402

pkg = pkgload.load()
from importlib import import_module  # noqa: E402

ve = import_module(pkg.__name__ + ".vectorized_env")
ppo_mod = import_module(pkg.__name__ + ".ppo")
DEV = "cuda:0"
fused = "torch" not in sys.argv[1:]
env = ve.FormationEnv({"num_formation": 1000, "num_agents_per_formation": 5, "goal_in_obs": True},
                      device=DEV, seed=2, reset_mode="philox")
m = ppo_mod.PPO(env, ppo_mod.PPOConfig(), seed=3, use_graph=not fused, use_fused=fused)
with torch.no_grad():
    m.collector.collect()
flat0 = m.policy.flat.clone()
st = m.train()
torch.cuda.synchronize()
d = (m.policy.flat - flat0)
print(("fused" if fused else "torch"), os.path.basename(os.environ.get("FENV_LIB_OVERRIDE", "in-tree")),
      {k: round(v, 10) for k, v in st.items()}, "log_std", m.policy.flat[-2:].tolist(),
      "max moved", round(d.abs().max().item(), 4), flush=True)
torch.save(m.policy.flat.cpu(), f"/tmp/refcfg_{'fused' if fused else 'torch'}_"
           f"{os.path.basename(os.environ.get('FENV_LIB_OVERRIDE', 'intree'))}.pt")
