"""Host cost (us, median of 200) of each call bench.py's timed region makes before and between its
launches, on a small env (4,096 x 5: the launches are short, so the queue never fills and no call
blocks).  Each call is timed alone with perf_counter, after a synchronize, like the region's first
launch (cold-ish), and back to back (warm)."""
import ctypes
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pkgload  # noqa: E402

pkg = pkgload.load()
from importlib import import_module  # noqa: E402

venv = import_module(pkg.__name__ + ".vectorized_env")
flib = import_module(pkg.__name__ + "._lib")
pdist = import_module(pkg.__name__ + ".distributed")
dev = torch.device("cuda", 0)
F, N, T = 4096, 5, 10
env = venv.FormationEnv({"num_formation": F, "num_agents_per_formation": N, "goal_in_obs": True},
                        log=False, device=dev, seed=0, reset_mode="philox")
A = env.num_envs
acts = torch.rand((T, A, 2), device=dev) * 2 - 1
obs = torch.empty((T, A, 8), device=dev)
rew = torch.empty((T, A), device=dev)
done = torch.empty((T, A), dtype=torch.bool, device=dev)
part = torch.zeros((env.partial_count(), 2), device=dev)
red = torch.zeros(2, dtype=torch.float64, device=dev)
main = torch.cuda.current_stream(dev)
side = torch.cuda.Stream(dev)
L = flib.lib()
vp = ctypes.c_void_p
args = (env._h, T, vp(acts.data_ptr()), vp(obs.data_ptr()), vp(rew.data_ptr()),
        vp(done.data_ptr()))
sp, ssp = vp(main.cuda_stream), vp(side.cuda_stream)
npart = env.partial_count()
ev_t = torch.cuda.Event(enable_timing=True)
ev_n = torch.cuda.Event()
for e in (ev_t, ev_n):
    e.record(main)
stats = pdist.StatsReducer(2, dev, stream=side)
fn = L.fenv_rollout

calls = {
    "event_record_timing": lambda: ev_t.record(main),
    "event_record_plain": lambda: ev_n.record(main),
    "event_query": lambda: ev_n.query(),
    "wait_event": lambda: side.wait_event(ev_n),
    "fenv_rollout_ctypes": lambda: fn(*args, None, sp),
    "fenv_rollout_ctypes_partial": lambda: fn(*args, vp(part.data_ptr()), sp),
    "fenv_reduce_partials_ctypes": lambda: L.fenv_reduce_partials(vp(part.data_ptr()), npart,
                                                                   vp(red.data_ptr()), ssp),
    "stats_submit_world1": lambda: stats.submit(red, stream=side),
    "stream_context": lambda: torch.cuda.stream(side).__enter__() and None,
    "perf_counter": lambda: time.perf_counter(),
}


def timeit(f, cold):
    out = []
    for _ in range(200):
        if cold:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        f()
        out.append((time.perf_counter() - t0) * 1e6)
    torch.cuda.synchronize()
    return statistics.median(out)


res = {}
for name, f in calls.items():
    if name == "stream_context":
        def f():  # noqa: E731 -- enter and leave, as `with torch.cuda.stream(side):` does
            with torch.cuda.stream(side):
                pass
    for _ in range(20):
        f()
    torch.cuda.synchronize()
    res[name] = {"after_sync_us": timeit(f, True), "back_to_back_us": timeit(f, False)}
print(json.dumps(res, indent=1))
