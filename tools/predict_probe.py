"""Per-call time of MlpPolicy.predict (SB3's ``model.predict(obs, deterministic=True)``,
visualize_policy.py:16) on numpy observations, and of the predict + env.step loop the reference's
playback runs (visualize_policy.py:16-18), at B = 5 (playback: one formation) and 5,000 (config 0).
Median of many calls (us).
    python tools/predict_probe.py [calls]   -> one JSON line per batch size
"""
import json
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pkgload  # noqa: E402

pkg = pkgload.load()
from importlib import import_module  # noqa: E402

venv = import_module(pkg.__name__ + ".vectorized_env")
pol = import_module(pkg.__name__ + ".policy")
CALLS = int(sys.argv[1]) if len(sys.argv) > 1 else 300
dev = torch.device("cuda", 0)


def med(fn, n=CALLS):
    for _ in range(10):
        fn()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(1e6 * statistics.median(ts), 2)


for F in (1, 1000):
    env = venv.FormationEnv({"num_formation": F, "num_agents_per_formation": 5,
                             "goal_in_obs": True}, log=False, device=dev, seed=0,
                            reset_mode="philox")
    model = pol.MlpPolicy(8, device=dev, seed=0)
    obs = env.reset()
    plain = obs.copy()
    # the same actions as forward(): bit for bit
    ref = model.forward(torch.from_numpy(plain).to(dev), deterministic=True,
                        offset=12345)["clipped"].cpu().numpy()
    model._offset = 12345
    got, _ = model.predict(plain, deterministic=True)
    out = {"B": env.num_envs, "predict_equals_forward": bool(np.array_equal(got, ref))}
    out["predict_env_obs_us"] = med(lambda: model.predict(obs, deterministic=True))
    out["predict_plain_obs_us"] = med(lambda: model.predict(plain, deterministic=True))
    state = {"o": obs}

    def loop():
        a, _ = model.predict(state["o"], deterministic=True)
        state["o"], _, _, _ = env.step(a)

    out["predict_step_loop_us"] = med(loop)
    print(json.dumps(out), flush=True)
    env.release()
