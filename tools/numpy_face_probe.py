"""Per-step time of the numpy face against the pinned-mirror path it replaced.

FormationEnv.step(np.ndarray) (vectorized_env.py) runs the kernel on device-mapped host arrays
(fenv_host_alloc): the actions are read and obs / reward / done written in place, one launch and
a synchronize per step.  Until round 5 it copied the actions host -> device and the three
outputs device -> host through torch pinned mirrors.  Median of many calls at the sizes given:
  full       env.step(numpy)   (outputs checked bit for bit against a twin on the device face)
  kernel     env.step_tensor(device actions) + synchronize
  legacy     the replaced path: numpy -> pinned -> device action copy, step_tensor, three output
             copies into pinned mirrors, synchronize
  hybrid     actions read in place, outputs to a device block and back in one DMA copy
    python tools/numpy_face_probe.py [formations] [agents] [calls]   -> one JSON line
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
F = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
N = int(sys.argv[2]) if len(sys.argv) > 2 else 5
CALLS = int(sys.argv[3]) if len(sys.argv) > 3 else 400
dev = torch.device("cuda", 0)
cfg = {"num_formation": F, "num_agents_per_formation": N, "goal_in_obs": True}
env = venv.FormationEnv(cfg, log=False, device=dev, seed=0, reset_mode="philox")
twin = venv.FormationEnv(cfg, log=False, device=dev, seed=0, reset_mode="philox")
A, D = env.num_envs, env.obs_dim
rng = np.random.default_rng(3)
acts = [rng.uniform(-1, 1, (A, 2)).astype(np.float32) for _ in range(4)]
stream = torch.cuda.current_stream(dev)


def med(fn, n=CALLS):
    for _ in range(10):
        fn()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return 1e6 * statistics.median(ts)


out = {"formations": F, "agents": N, "calls": CALLS}
env.reset()
twin.reset_tensor()
bad = 0
for s in range(40):
    a = acts[s & 3]
    o, r, d, _ = env.step(a)
    to, tr, td = twin.step_tensor(torch.from_numpy(a).to(dev))
    bad += int(not (np.array_equal(o.view(np.uint32), to.cpu().numpy().view(np.uint32))
                    and np.array_equal(r.view(np.uint32), tr.cpu().numpy().view(np.uint32))
                    and np.array_equal(d, td.cpu().numpy())))
out["mismatched_steps"] = bad
k = [0]


def full():
    env.step(acts[k[0] & 3])
    k[0] += 1


out["full_us"] = med(full)
act_dev = torch.from_numpy(acts[0]).to(dev)


def kern():
    twin.step_tensor(act_dev)
    stream.synchronize()


out["kernel_us"] = med(kern)
pin = {n: torch.zeros(s, dtype=t, pin_memory=True)
       for n, s, t in (("act", (A, 2), torch.float32), ("obs", (A, D), torch.float32),
                       ("rew", (A,), torch.float32), ("done", (A,), torch.bool))}
act_buf = torch.zeros((A, 2), dtype=torch.float32, device=dev)


def legacy():
    pin["act"].numpy()[...] = acts[k[0] & 3]
    act_buf.copy_(pin["act"], non_blocking=True)
    twin.step_tensor(act_buf)
    pin["obs"].copy_(twin.obs_dev, non_blocking=True)
    pin["rew"].copy_(twin.rew_dev, non_blocking=True)
    pin["done"].copy_(twin.done_dev, non_blocking=True)
    stream.synchronize()
    k[0] += 1


out["legacy_us"] = med(legacy)

# hybrid: the kernel reads the actions in place (host block) and writes obs / reward / done to a
# device block laid out like the host block; one DMA copies the three back
import ctypes  # noqa: E402
hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                               ctypes.c_void_p]
flib = import_module(pkg.__name__ + "._lib")
hb = env._ensure_host()
o_obs = hb.obs.ctypes.data - hb.act.ctypes.data
o_rew = hb.rew.ctypes.data - hb.act.ctypes.data
o_done = hb.done.ctypes.data - hb.act.ctypes.data
span = o_done + A - o_obs
dblk = torch.empty(o_done + A + 256, dtype=torch.uint8, device=dev)
db = dblk.data_ptr()
L = flib.lib()


def hybrid():
    np.copyto(hb.act, acts[k[0] & 3])
    st = env._stream()
    flib.check(L.fenv_step(env._h, hb.dev("act"), ctypes.c_void_p(db + o_obs),
                           ctypes.c_void_p(db + o_rew), ctypes.c_void_p(db + o_done), st), "step")
    assert hip.hipMemcpyAsync(hb.obs.ctypes.data, db + o_obs, span, 2, st) == 0
    stream.synchronize()
    k[0] += 1


out["hybrid_us"] = med(hybrid)
out["full_over_legacy"] = out["full_us"] / out["legacy_us"]
out["pcie_gbs_full"] = A * (8 + 4 * D + 4 + 1) / out["full_us"] / 1e3
print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in out.items()}),
      flush=True)
env.release()
twin.release()
