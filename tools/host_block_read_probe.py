"""CPU access speed of the numpy faces' device-mapped host arrays (fenv_host_alloc: coherent
host memory) against ordinary numpy memory, at config 3's obs size (168 MB): sum, copy out, and a
fill of the action array.  Min of 5 after one warm call (ms).
    python tools/host_block_read_probe.py   -> one JSON line
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401

import pkgload  # noqa: E402

pkg = pkgload.load()
from importlib import import_module  # noqa: E402

venv = import_module(pkg.__name__ + ".vectorized_env")
env = venv.FormationEnv({"num_formation": 1048576, "num_agents_per_formation": 5,
                         "goal_in_obs": True}, log=False, device="cuda:0", seed=0,
                        reset_mode="philox")
o = env.reset()
c = o.copy()
act_plain = np.empty_like(env._host.act)


def t(f, n=5):
    f()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return round(min(ts) * 1e3, 3)


out = {"obs_mb": o.nbytes / 1e6,
       "sum_block_ms": t(lambda: o.sum()), "sum_plain_ms": t(lambda: c.sum()),
       "copy_block_ms": t(lambda: o.copy()), "copy_plain_ms": t(lambda: c.copy()),
       "fill_act_block_ms": t(lambda: np.copyto(env._host.act, 0.5)),
       "fill_act_plain_ms": t(lambda: np.copyto(act_plain, 0.5))}
print(json.dumps(out), flush=True)
env.release()
