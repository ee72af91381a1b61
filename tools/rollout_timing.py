"""Config-2 timing (65,536 formations x 10 agents, n_steps = 10): policy_forward alone, the fused
rollout kernel (fenv_policy_rollout) and the per-step collector, with HIP events on the launch
stream.  Prints one line each; FLOP counts are the algorithmic 18,816 per agent-step (+9,344 per
agent for the last value in a rollout)."""
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
F = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
N = int(sys.argv[2]) if len(sys.argv) > 2 else 10
T = 10
dev = torch.device("cuda", 0)
A = F * N
PEAK = 157.3


def timed(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    best = None
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / reps
        best = ms if best is None else min(best, ms)
    return best


pol = pol_mod.MlpPolicy(8, device=dev, seed=0)
obs = torch.rand((A, 8), device=dev) * 2 - 1
out = dict(mu=torch.empty((A, 2), device=dev), value=torch.empty(A, device=dev),
           action=torch.empty((A, 2), device=dev), log_prob=torch.empty(A, device=dev),
           clipped=torch.empty((A, 2), device=dev))
ms = timed(lambda: pol.forward(obs, out=out, seed=0, offset=0), 20)
tf = 18816.0 * A / (ms * 1e-3) / 1e12
print(f"policy_forward A={A}: {ms*1e3:.1f} us  {tf:.1f} TFLOP/s  {tf/PEAK*100:.1f}% fp32 MFMA",
      flush=True)
cfg = {"num_formation": F, "num_agents_per_formation": N, "goal_in_obs": True}
for fused in (True, False):
    env = venv.FormationEnv(cfg, log=False, device=dev, seed=1, reset_mode="philox")
    buf = ro.RolloutBuffer(T, A, 8, dev)
    col = ro.RolloutCollector(env, pol, buf, seed=0, fused=fused)
    ms = timed(col.collect, 5)
    flop = A * (T * 18816.0 + 9344.0)
    tf = flop / (ms * 1e-3) / 1e12
    print(f"collect fused={fused} F={F} N={N} T={T}: {ms*1e3:.1f} us/rollout  "
          f"{A*T/(ms*1e-3):.3e} agent-steps/s  {tf:.1f} TFLOP/s  {tf/PEAK*100:.1f}% fp32 MFMA",
          flush=True)
