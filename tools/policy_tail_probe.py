"""Is the fused policy rollout (k_policy_rollout) paying for its last, partial round of
wave-units?  Its persistent grid holds 3,072 waves (768 workgroups x 4); a wave-unit is 6
formations at N = 10.  Times the fused kernel (bench.policy_rollout_bench, warm) at F = 55,296
(exactly 3 rounds), 65,536 (BASELINE config 2: 3.56 rounds) and 73,728 (exactly 4 rounds)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
import pkgload  # noqa: E402

pkg = pkgload.load()
dev = torch.device("cuda", 0)
for F in (55296, 65536, 73728, 65536):
    r = bench.policy_rollout_bench(pkg.__name__, dev, F, 10, 10)
    ms = r["rollout_kernel_ms"]
    print(f"F {F:6d}  units {F / 6:8.1f}  rounds {F / 6 / 3072:5.2f}  kernel {ms * 1e3:7.1f} us  "
          f"{F * 10 * 10 / (ms * 1e-3):.3e} agent-steps/s", flush=True)
