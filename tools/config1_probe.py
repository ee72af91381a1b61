"""Where config 1's time goes (4,096 x 5, latency-bound): launch time vs T, and with outputs
dropped through the C ABI (obs / reward / done pointers NULL), HIP events over 2,000 launches."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pkgload  # noqa: E402

pkg = pkgload.load()
from importlib import import_module  # noqa: E402

venv = import_module(pkg.__name__ + ".vectorized_env")
_lib = import_module(pkg.__name__ + "._lib")
dev = torch.device("cuda", 0)
F, N = int(os.environ.get("F", 4096)), int(os.environ.get("N", 5))
env = venv.FormationEnv({"num_formation": F, "num_agents_per_formation": N, "goal_in_obs": True},
                        device=dev, seed=0, reset_mode="philox")
A, L = env.num_envs, _lib.lib()
TM = 20
acts = torch.rand((TM, A, 2), device=dev) * 2 - 1
obs = torch.empty((TM, A, 8), device=dev)
rew = torch.empty((TM, A), device=dev)
done = torch.empty((TM, A), dtype=torch.bool, device=dev)
P = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())  # noqa: E731
st = _lib.current_stream(dev)


def timed(T, o, r, d, n=2000):
    f = lambda: L.fenv_rollout(env._h, T, P(acts), P(o), P(r), P(d), None, st)  # noqa: E731
    for _ in range(50):
        f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        f()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


for T in (1, 2, 5, 10, 20):
    print(f"F={F} N={N} T={T:2d}: all outputs {timed(T, obs, rew, done):6.2f} us | no obs "
          f"{timed(T, None, rew, done):6.2f} | no rew/done {timed(T, obs, None, None):6.2f} | "
          f"nothing {timed(T, None, None, None):6.2f}", flush=True)
