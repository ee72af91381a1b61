"""Same-box A/B of the fused policy rollout (BASELINE config 2, 65,536 x 10): bench.py's
policy_rollout_bench (>= 300 ms warm-up, then the kernel alone over 10 rollouts with HIP events),
one line per library (FENV_LIB_OVERRIDE selects it; the caller loops over build_variants/*.so)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
import pkgload  # noqa: E402

pkg = pkgload.load()
dev = torch.device("cuda", 0)
lib = os.path.basename(os.environ.get("FENV_LIB_OVERRIDE", "in-tree"))
r = bench.policy_rollout_bench(pkg.__name__, dev, 65536, 10, 10)
print(f"{lib:36s} policy_rollout kernel {r['rollout_kernel_ms'] * 1e3:7.1f} us  collect "
      f"{r['value']:.3e} agent-steps/s  policy_forward {r['policy_kernel_ms'] * 1e3:6.1f} us",
      flush=True)
