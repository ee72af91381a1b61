"""Same-box A/B of the env rollout kernels at BASELINE configs 1, 3 and 4 (bench.py's
env_config_bench: fused 10-step rollouts, HIP events): one line per library, the library chosen
by FENV_LIB_OVERRIDE (the caller loops over build_variants/*.so)."""
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
out = []
for name, F, N, launches in (("c1", 4096, 5, 1000), ("c4", 16384, 64, 100), ("c3", 1 << 20, 5, 100)):
    r = bench.env_config_bench(pkg.__name__, dev, F, N, launches)
    out.append(f"{name} {r['avg_kernel_ms'] * 1e3:7.2f} us")
r = bench.env_config_bench(pkg.__name__, dev, 1 << 20, 5, 100, T=1)  # the fenv_step face
out.append(f"c3/T1 {r['avg_kernel_ms'] * 1e3:6.2f} us")
print(f"{lib:36s} " + "  ".join(out), flush=True)
