"""Where does RolloutCollector.collect spend the time beyond the fused kernel?  BASELINE config 2
(65,536 x 10).  Prints per collect: wall time of 10 back-to-back collects, host time to issue
one collect, and HIP-event device time of the fused launch with and without the GAE buffers."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pkgload  # noqa: E402

pkg = pkgload.load()
from importlib import import_module  # noqa: E402

venv = import_module(pkg.__name__ + ".vectorized_env")
pol_mod = import_module(pkg.__name__ + ".policy")
ro = import_module(pkg.__name__ + ".rollout")
dev = torch.device("cuda", 0)
cfg = {"num_formation": 65536, "num_agents_per_formation": 10, "goal_in_obs": True}
env = venv.FormationEnv(cfg, log=False, device=dev, seed=1, reset_mode="philox")
pol = pol_mod.MlpPolicy(8, device=dev, seed=0)
buf = ro.RolloutBuffer(10, env.num_envs, 8, dev)
col = ro.RolloutCollector(env, pol, buf, seed=0)
for _ in range(3):
    col.collect()
torch.cuda.synchronize()
R = 20
host = []
t0 = time.perf_counter()
for _ in range(R):
    h0 = time.perf_counter()
    col.collect()
    host.append(time.perf_counter() - h0)
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / R
full = dict(obs=buf.observations, mu=buf.mu, action=buf.actions, clipped=buf.clipped,
            value=buf.values, log_prob=buf.log_probs, reward=buf.rewards,
            episode_start=buf.episode_starts, done=buf.dones, last_done=col.last_episode_starts,
            last_obs=col.last_obs, last_value=col._last_values)


def dev_ms(bufs):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(3):
        env.policy_rollout(pol.flat, 10, bufs, seed=0, offset=5000 + 10 * r)
    a.record()
    for r in range(R):
        env.policy_rollout(pol.flat, 10, bufs, seed=0, offset=1000 + 10 * r)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / R


k_only = dev_ms(full)
k_gae = dev_ms(dict(full, advantage=buf.advantages, ret=buf.returns))
# collect() again, now with events as well as wall time, and the direct calls with wall time
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize()
t0 = time.perf_counter()
a.record()
for _ in range(R):
    col.collect()
b.record()
torch.cuda.synchronize()
wall2 = (time.perf_counter() - t0) / R
ev2 = a.elapsed_time(b) / R
gb = dict(full, advantage=buf.advantages, ret=buf.returns)
torch.cuda.synchronize()
t0 = time.perf_counter()
for r in range(R):
    env.policy_rollout(pol.flat, 10, gb, seed=0, offset=9000 + 10 * r)
torch.cuda.synchronize()
wall3 = (time.perf_counter() - t0) / R
print(f"collect wall {wall * 1e6:7.1f} us   host issue {sorted(host)[R // 2] * 1e6:7.1f} us (median)   "
      f"fused kernel {k_only * 1e3:7.1f} us   kernel + GAE {k_gae * 1e3:7.1f} us   "
      f"collect again: wall {wall2 * 1e6:7.1f} events {ev2 * 1e3:7.1f}   direct calls wall "
      f"{wall3 * 1e6:7.1f} us", flush=True)
