"""which library faults when a process that made the PPO update's cooperative
launch exits under rocprofv3?  Runs one fused PPO update (the split kernel's
hipLaunchCooperativeKernel) and, from a Python atexit hook -- which runs before the C exit
handlers where the crash happens -- writes this process's /proc/self/maps next to the profiler
output, so the unsymbolized PCs glog prints can be
mapped to library + offset afterwards (tools/symbolize_maps.py).

    rocprofv3 --kernel-trace --stats -d OUT -o p -- python3 tools/coop_exit_probe.py OUT [release]

`release` destroys the env and the PPO object before exit (the crash happens either way?)."""
import atexit
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "coop_exit")
os.makedirs(OUT, exist_ok=True)


@atexit.register
def _dump_maps():
    with open("/proc/self/maps") as f, open(os.path.join(OUT, f"maps_{os.getpid()}.txt"), "w") as o:
        o.write(f.read())


import torch  # noqa: E402

import pkgload  # noqa: E402

pkg = pkgload.load()
from importlib import import_module  # noqa: E402

venv = import_module(pkg.__name__ + ".vectorized_env")
ppo = import_module(pkg.__name__ + ".ppo")
env = venv.FormationEnv({"num_formation": 1000, "num_agents_per_formation": 5,
                         "goal_in_obs": True}, log=False, device="cuda:0", seed=0,
                        reset_mode="philox")
m = ppo.PPO(env, ppo.PPOConfig(), seed=0)
with torch.no_grad():
    m.collector.collect()
m.train()
torch.cuda.synchronize()
print(f"pid {os.getpid()} fused={m.use_fused} update done", flush=True)
if len(sys.argv) > 2 and sys.argv[2] == "release":
    env.release()
    del m, env
