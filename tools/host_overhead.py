"""Host-side cost of one launch through each layer (GPU box): FormationEnv.rollout (Python checks
+ ctypes), the bare C-ABI call, a torch event record, torch.cuda.current_stream.  A tiny env so
the GPU never holds the host back (launches queue asynchronously)."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pkgload  # noqa: E402

pkg = pkgload.load()
from importlib import import_module  # noqa: E402

venv = import_module(pkg.__name__ + ".vectorized_env")
_lib = import_module(pkg.__name__ + "._lib")
dev = torch.device("cuda", 0)
env = venv.FormationEnv({"num_formation": 64, "num_agents_per_formation": 5, "goal_in_obs": True},
                        device=dev, seed=0, reset_mode="philox")
A, T = env.num_envs, 10
acts = torch.zeros((T, A, 2), device=dev)
obs = torch.empty((T, A, 8), device=dev)
rew = torch.empty((T, A), device=dev)
done = torch.empty((T, A), dtype=torch.bool, device=dev)
part = torch.zeros((env.partial_count(), 2), device=dev)


def per_call(fn, n=2000):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    el = time.perf_counter() - t0
    torch.cuda.synchronize()
    return el / n * 1e6


L = _lib.lib()
ptrs = [ctypes.c_void_p(t.data_ptr()) for t in (acts, obs, rew, done)]
st = _lib.current_stream(dev)
ev = torch.cuda.Event(enable_timing=True)
print(f"env.rollout (checks + ctypes + launch): {per_call(lambda: env.rollout(acts, obs, rew, done)):.1f} us")
print(f"env.rollout with partial:               {per_call(lambda: env.rollout(acts, obs, rew, done, partial=part)):.1f} us")
print(f"bare fenv_rollout C call:               {per_call(lambda: L.fenv_rollout(env._h, T, *ptrs, None, st)):.1f} us")
print(f"torch.cuda.Event.record:                {per_call(lambda: ev.record()):.1f} us")
print(f"torch.cuda.current_stream:              {per_call(lambda: torch.cuda.current_stream(dev).cuda_stream):.1f} us")
print(f"env._check_out x3:                      {per_call(lambda: [env._check_out('o', obs, (T, A, 8), torch.float32), env._check_out('r', rew, (T, A), torch.float32), env._check_out('d', done, (T, A), torch.bool)]):.1f} us")
