"""Diagnose tests/test_gpu_parity.py::test_metrics_and_partials[500-5] (round 3: the partial-record
sum came out 6.3 % off the oracle's reward sum once).  Repeats the test's exact sequence in one
process and, each time, separates the candidates: are the rewards wrong (vs the C oracle, per
step), or are the per-group {reward, done} records wrong (vs the same group sums of the kernel's
own rewards, per launch)?"""
import os
import sys

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import pkgload  # noqa: E402
from oracle import COracleEnv, synth_actions  # noqa: E402

pkg = pkgload.load()
from importlib import import_module  # noqa: E402

venv = import_module(pkg.__name__ + ".vectorized_env")
DEV = "cuda:0"
F, N = 500, 5
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
for rep in range(reps):
    env = venv.FormationEnv({"num_formation": F, "num_agents_per_formation": N, "goal_in_obs": True},
                            device=DEV, seed=21, max_steps=3)
    ref = COracleEnv(F, N, True, 21, max_steps=3)
    env.reset()
    ref.reset()
    acts = np.stack([synth_actions(4, k, F * N, 1.0) for k in range(8)])
    npart = env.partial_count()
    partial = torch.zeros((npart, 2), dtype=torch.float32, device=DEV)
    obs, rew, done = env.rollout(torch.from_numpy(acts).to(DEV), partial=partial)
    torch.cuda.synchronize()
    r = rew.cpu().numpy()
    bad_steps = []
    rs = 0.0
    for k in range(8):
        _, rr, rd, _ = ref.step(acts[k])
        rs += rr.astype(np.float64).sum()
        if not np.array_equal(r[k].view(np.uint32), rr.view(np.uint32)):
            bad_steps.append((k, int((r[k] != rr).sum())))
    sums = env.reduce_partials(partial).cpu().numpy()
    # the records: one per group of 4 formation-waves (12 formations each at N = 5 -> 240 agents)
    per = 4 * (64 // N) * N
    own = np.array([r[:, g * per:(g + 1) * per].astype(np.float64).sum() for g in range(npart)])
    recs = partial.cpu().numpy()[:, 0].astype(np.float64)
    print(f"rep {rep}: kernel {env.rollout_kernel_name(5)}, records {npart}, record sum "
          f"{sums[0]:.6f}, oracle sum {rs:.6f}, kernel-reward sum {r.astype(np.float64).sum():.6f}, "
          f"reward mismatches {bad_steps}, records vs own group sums max diff "
          f"{np.abs(recs - own).max():.4f} at groups {np.nonzero(np.abs(recs - own) > 1e-2 * np.abs(own).max())[0].tolist()}",
          flush=True)
    env.release()
