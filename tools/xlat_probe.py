"""Headline-gap probe: fused config-3 rollouts (1,048,576 x 5, D = 8, Philox) in
footprint shapes that the round-2 probes showed run at different rates, one shape per process so
a rocprofv3 --pmc pass attributes its counters to that shape alone.

  t10      T = 10 launches, all into ONE 10-plane buffer set (the bench's shape, ~2.5 GB per launch)
  t4same   T = 4 launches, all into one 4-plane buffer set (~1 GB rewritten per launch)
  t4of10   T = 4, 4, 2 launches walking the planes of one 10-plane set (same bytes as t10)
  t10alt   T = 10 launches alternating between TWO 10-plane sets (5 GB reuse distance)

Prints one JSON line: microseconds per step from HIP events around each launch (on the launch
stream), the algorithmic GB/s, and the fraction of the 8 TB/s spec.  Usage:
    python tools/xlat_probe.py CASE [--launches K]
"""
import argparse
import json
import os
import sys

ROOT = os.environ.get("GRAFT_REPO_ROOT",
                      os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import pkgload  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("case", choices=["t10", "t4same", "t4of10", "t10alt"])
ap.add_argument("--launches", type=int, default=24)
ap.add_argument("--alloc", choices=["torch", "onechunk", "contig"], default="torch",
                help="onechunk: every plane of a set carved from one torch allocation; contig: "
                     "each buffer from hipExtMallocWithFlags(hipDeviceMallocContiguous)")
args = ap.parse_args()

pkg = pkgload.load()
from importlib import import_module  # noqa: E402

venv = import_module(pkg.__name__ + ".vectorized_env")
dev = torch.device("cuda", 0)
F, N, D = 1 << 20, 5, 8
A = F * N
env = venv.FormationEnv({"num_formation": F, "num_agents_per_formation": N, "goal_in_obs": True},
                        log=False, device=dev, seed=0, reset_mode="philox")
env.reset_tensor()


class _Raw:
    """A hipExtMallocWithFlags buffer exposed to torch through __cuda_array_interface__."""
    hip = None

    def __init__(self, shape, dtype, flags):
        import ctypes
        if _Raw.hip is None:
            _Raw.hip = ctypes.CDLL("libamdhip64.so")
        n = 1
        for d in shape:
            n *= d
        esz = torch.empty((), dtype=dtype).element_size()
        self.p = ctypes.c_void_p()
        rc = _Raw.hip.hipExtMallocWithFlags(ctypes.byref(self.p), ctypes.c_size_t(n * esz),
                                           ctypes.c_uint(flags))
        if rc != 0:
            raise RuntimeError(f"hipExtMallocWithFlags rc={rc}")
        typestr = {torch.float32: "<f4", torch.bool: "|b1"}[dtype]
        self.__cuda_array_interface__ = {"shape": tuple(shape), "typestr": typestr,
                                         "data": (self.p.value, False), "version": 2}


_keep = []


def raw_tensor(shape, dtype):
    r = _Raw(shape, dtype, 0x4)  # hipDeviceMallocContiguous
    _keep.append(r)
    return torch.as_tensor(r, device=dev)


def bufset(P):
    if args.alloc == "contig":
        act = raw_tensor((P, A, 2), torch.float32)
        act.uniform_(-1, 1)
        return (act, raw_tensor((P, A, D), torch.float32), raw_tensor((P, A), torch.float32),
                raw_tensor((P, A), torch.bool))
    if args.alloc == "onechunk":
        per = A * (2 * 4 + D * 4 + 4 + 1) + 4 * 4096
        raw = torch.empty(P * per, dtype=torch.uint8, device=dev)
        # planes of one stream contiguous (the API's [T, A, ...] layout) inside the chunk
        o = 0
        views = []
        for shape, dt, esz in (((P, A, 2), torch.float32, 4), ((P, A, D), torch.float32, 4),
                               ((P, A), torch.float32, 4), ((P, A), torch.bool, 1)):
            n = 1
            for s in shape:
                n *= s
            nbytes = (n * esz + 4095) // 4096 * 4096
            views.append(raw[o:o + n * esz].view(dt).view(shape))
            o += nbytes
        act = views[0]
        act.uniform_(-1, 1)
        return tuple(views)
    act = torch.rand((P, A, 2), device=dev) * 2 - 1
    return (act, torch.empty((P, A, D), device=dev), torch.empty((P, A), device=dev),
            torch.empty((P, A), dtype=torch.bool, device=dev))


if args.case == "t10":
    sets = [bufset(10)]
    plan = [(0, 0, 10)]
elif args.case == "t4same":
    sets = [bufset(4)]
    plan = [(0, 0, 4)]
elif args.case == "t4of10":
    sets = [bufset(10)]
    plan = [(0, 0, 4), (0, 4, 8), (0, 8, 10)]
else:
    sets = [bufset(10), bufset(10)]
    plan = [(0, 0, 10), (1, 0, 10)]

stream = torch.cuda.current_stream(dev)


def launch(i):
    s, lo, hi = plan[i % len(plan)]
    a, o, r, d = sets[s]
    env.rollout(a[lo:hi], o[lo:hi], r[lo:hi], d[lo:hi])
    return hi - lo


for i in range(2 * len(plan)):  # warm-up
    launch(i)
torch.cuda.synchronize()
K = max(args.launches // len(plan), 1) * len(plan)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(K + 1)]
steps = []
ev[0].record(stream)
for i in range(K):
    steps.append(launch(i))
    ev[i + 1].record(stream)
torch.cuda.synchronize()
ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(K)]
tot_ms, tot_steps = sum(ms), sum(steps)
# algorithmic bytes: 45 B per agent-step + 20 B per agent per launch
nbytes = sum(A * (45 * t + 16) + F * 20 for t in steps)
gbs = nbytes / (tot_ms * 1e-3) / 1e9
print(json.dumps({"case": args.case, "alloc": args.alloc, "launches": K,
                  "us_per_step": tot_ms * 1e3 / tot_steps, "GBps": gbs, "frac_of_8TBps": gbs / 8000,
                  "launch_us_min": min(ms) * 1e3, "launch_us_max": max(ms) * 1e3}), flush=True)
