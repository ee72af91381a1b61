"""Fused rollout length sweep at BASELINE config 3 (1,048,576 x 5): device time per launch and per
step for several launch lengths T (HIP-graph replays, bench.env_config_bench), ROUNDS rounds in
rotating order."""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
import pkgload  # noqa: E402

pkg = pkgload.load()
dev = torch.device("cuda", 0)
Ts = [int(t) for t in os.environ.get("TS", "10,8,7,6,5,4").split(",")]
for rnd in range(int(os.environ.get("ROUNDS", "3"))):
    order = Ts[rnd % len(Ts):] + Ts[:rnd % len(Ts)]
    for T in order:
        r = bench.env_config_bench(pkg.__name__, dev, 1 << 20, 5, max(20, 200 // T), T=T)
        us = r["avg_kernel_ms"] * 1e3
        print(f"round {rnd} T={T:2d}: {us:7.1f} us per launch = {us / T:5.1f} us per step, "
              f"{5242880 * T / (us * 1e-6):.3e} agent-steps/s, {r['hbm_frac']:.3f} of spec "
              f"({r['algorithmic_bytes_per_launch'] / 5242880 / T:.1f} B per agent-step)",
              flush=True)
