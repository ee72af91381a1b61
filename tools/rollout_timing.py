"""Config-2 timing (65,536 formations x 10 agents, n_steps = 10): policy_forward alone, the fused
rollout kernel (fenv_policy_rollout) and the per-step collector, with HIP events on the launch
stream.  Prints one line each: fp32-equivalent FLOP are the algorithmic 18,816 per agent-step
(+9,344 per agent for the last value in a rollout); the f16 MFMA rate counts the split-f16
MFMAs actually issued (3 per fp32 product, layer-1 k padded to 16)."""
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
F16_PEAK = 2516.6  # dense f16 MFMA TF/s (MI355X_MICROARCH.md: 16 x the 157.3 TF fp32 rate)
# split-f16 MFMA work actually issued (policy_device.h): 56 x 32x32x16 MFMAs per 32-agent tile
F16_FLOP_STEP = 56 * 32768 / 32      # per agent-step (actor + critic)
F16_FLOP_VALUE = 28 * 32768 / 32     # per agent, critic only (last value of a rollout)


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
mf = F16_FLOP_STEP * A / (ms * 1e-3) / 1e12
print(f"policy_forward A={A}: {ms*1e3:.1f} us  {tf:.1f} fp32-equiv TFLOP/s  "
      f"f16 MFMA {mf:.0f} TF/s ({mf/F16_PEAK*100:.1f}%)", flush=True)
cfg = {"num_formation": F, "num_agents_per_formation": N, "goal_in_obs": True}
for fused in (True, False):
    env = venv.FormationEnv(cfg, log=False, device=dev, seed=1, reset_mode="philox")
    buf = ro.RolloutBuffer(T, A, 8, dev)
    col = ro.RolloutCollector(env, pol, buf, seed=0, fused=fused)
    ms = timed(col.collect, 5)
    tf = A * (T * 18816.0 + 9344.0) / (ms * 1e-3) / 1e12
    mf = A * (T * F16_FLOP_STEP + F16_FLOP_VALUE) / (ms * 1e-3) / 1e12
    print(f"collect fused={fused} F={F} N={N} T={T}: {ms*1e3:.1f} us/rollout  "
          f"{A*T/(ms*1e-3):.3e} agent-steps/s  {tf:.1f} fp32-equiv TFLOP/s  "
          f"f16 MFMA {mf:.0f} TF/s ({mf/F16_PEAK*100:.1f}%)", flush=True)
