"""Time one PPO iteration (collect + train) on the reference's default training config
(1000 formations x 5 agents, n_steps=10, SB3 defaults: batch 64, 10 epochs) and a large-batch one."""
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
for F, bs, epochs in ((1000, 64, 10), (65536, 65536, 10)):
    for graph, fused in ((False, False), (True, False), (False, True)):
        if fused and bs > 64:
            continue
        env = venv.FormationEnv({"num_formation": F, "num_agents_per_formation": 5,
                                 "goal_in_obs": True}, device=dev, seed=0, reset_mode="philox")
        cfg = ppo_mod.PPOConfig(batch_size=bs, n_epochs=epochs)
        m = ppo_mod.PPO(env, cfg, seed=0, use_graph=graph, use_fused=fused)
        for it in range(3):
            torch.cuda.synchronize()
            if not fused and not graph and it > 0 and F == 1000:
                break  # the eager loop is slow; one iteration is enough
            t0 = time.perf_counter()
            with torch.no_grad():
                m.collector.collect()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            st = m.train()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
        nb = -(-env.num_envs * 10 // bs) * epochs
        print(f"F={F} batch={bs} graph={graph} fused={fused}: collect {1e3*(t1-t0):.2f} ms, train {1e3*(t2-t1):.1f} ms "
              f"({nb} minibatches, {1e6*(t2-t1)/nb:.0f} us each), stats {st}", flush=True)
