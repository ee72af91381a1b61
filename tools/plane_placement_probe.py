"""Why do 4-step launches at config 3 stream at ~0.89 of the HBM spec in their own buffers
(tools/chunk_sweep.py) but not as 4-step pieces of a 10-step buffer (profiles/ab/r2_chunk_ab.txt)?
Times fused rollouts of T steps into views of larger rollout buffers: [T] = fresh T-plane
buffers, [lo:hi] = planes lo..hi-1 of 10-plane buffers (device time, HIP-graph replays)."""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
import pkgload  # noqa: E402

pkg = pkgload.load()
from importlib import import_module  # noqa: E402

venv = import_module(pkg.__name__ + ".vectorized_env")
dev = torch.device("cuda", 0)
F, N = 1 << 20, 5
A = F * N
env = venv.FormationEnv({"num_formation": F, "num_agents_per_formation": N, "goal_in_obs": True},
                        log=False, device=dev, seed=0, reset_mode="philox")
env.reset_tensor()


def bufs(P):
    return (torch.rand((P, A, 2), device=dev) * 2 - 1, torch.empty((P, A, 8), device=dev),
            torch.empty((P, A), device=dev), torch.empty((P, A), dtype=torch.bool, device=dev))


def time_views(views, reps=20):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for (a, o, r, d) in views:
            env.rollout(a, o, r, d)
    for _ in range(5):
        g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    steps = sum(v[0].shape[0] for v in views)
    return e0.elapsed_time(e1) / reps * 1e3 / steps  # us per step


b10 = bufs(10)
for rnd in range(2):
    b4 = bufs(4)
    cases = [
        ("fresh [4]", [b4]),
        ("[0:4] of 10", [tuple(x[0:4] for x in b10)]),
        ("[6:10] of 10", [tuple(x[6:10] for x in b10)]),
        ("[0:4]+[4:8]+[8:10] of 10", [tuple(x[0:4] for x in b10), tuple(x[4:8] for x in b10),
                                      tuple(x[8:10] for x in b10)]),
        ("[0:10] one launch", [b10]),
        ("fresh [4] x 3", [b4, b4, b4]),
    ]
    for name, views in cases:
        print(f"round {rnd} {name:28s} {time_views(views):6.1f} us per step", flush=True)
    del b4
    torch.cuda.empty_cache()
