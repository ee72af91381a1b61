"""Time policy_forward (config 2 batch: 655,360 agents) with HIP events; print fp32-equivalent TFLOP/s and the split-f16 MFMA rate."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pkgload  # noqa: E402

pkg = pkgload.load()
from importlib import import_module  # noqa: E402

pol_mod = import_module(pkg.__name__ + ".policy")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 655360
dev = torch.device("cuda", 0)
pol = pol_mod.MlpPolicy(8, device=dev, seed=0)
obs = torch.rand((B, 8), device=dev) * 2 - 1
out = dict(mu=torch.empty((B, 2), device=dev), value=torch.empty(B, device=dev),
           action=torch.empty((B, 2), device=dev), log_prob=torch.empty(B, device=dev),
           clipped=torch.empty((B, 2), device=dev))
for _ in range(20):
    pol.forward(obs, out=out, seed=0, offset=0)
torch.cuda.synchronize()
res = []
for rep in range(3):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(50)]
    for a, b in evs:
        a.record()
        pol.forward(obs, out=out, seed=0, offset=0)
        b.record()
    torch.cuda.synchronize()
    ms = sum(a.elapsed_time(b) for a, b in evs) / len(evs)
    res.append(ms)
ms = min(res)
tf = 18816.0 * B / (ms * 1e-3) / 1e12
print(f"{os.environ.get('FENV_LIB_OVERRIDE', 'libfenv.so')} B={B} policy {ms*1e3:.1f} us "
      f"{tf:.1f} fp32-equiv TFLOP/s, f16 MFMA {tf*57344/18816:.0f} TF/s "
      f"({tf*57344/18816/2516.6*100:.1f}% of dense f16 peak)", flush=True)
