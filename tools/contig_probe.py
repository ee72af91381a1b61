"""Is the config-3 rollout bound by address translation?  Times 10-step fenv_rollout calls (C ABI,
HIP events) into rollout buffers allocated three ways: by torch's caching allocator, by plain
hipMalloc, and by hipExtMallocWithFlags(hipDeviceMallocContiguous) (physically contiguous, so
the driver can map it with large fragments)."""
import ctypes
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import pkgload  # noqa: E402

pkg = pkgload.load()
from importlib import import_module  # noqa: E402

venv = import_module(pkg.__name__ + ".vectorized_env")
flib = import_module(pkg.__name__ + "._lib")
L = flib.lib()
hip = ctypes.CDLL("libamdhip64.so.7")  # the runtime torch already loaded (same soname)
hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
hip.hipFree.argtypes = [ctypes.c_void_p]
hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
dev = torch.device("cuda", 0)
F, N, T = 1 << 20, 5, 10
A = F * N
env = venv.FormationEnv({"num_formation": F, "num_agents_per_formation": N, "goal_in_obs": True},
                        log=False, device=dev, seed=0, reset_mode="philox")
env.reset_tensor()
src = torch.rand((T, A, 2), device=dev) * 2 - 1
sizes = [T * A * 8, T * A * 32, T * A * 4, T * A]


def alloc(kind):
    if kind == "torch":
        ts = [torch.empty(sz, dtype=torch.uint8, device=dev) for sz in sizes]
        return [t.data_ptr() for t in ts], ts
    ptrs = []
    for sz in sizes:
        p = ctypes.c_void_p()
        rc = (hip.hipMalloc(ctypes.byref(p), sz) if kind == "hipMalloc"
              else hip.hipExtMallocWithFlags(ctypes.byref(p), sz, 0x4))
        if rc != 0:
            raise RuntimeError(f"{kind} failed: {rc}")
        ptrs.append(p.value)
    return ptrs, None


def run(ptrs, reps=20):
    a, o, r, d = (ctypes.c_void_p(p) for p in ptrs)
    st = flib.current_stream(dev)
    for _ in range(5):
        flib.check(L.fenv_rollout(env._h, T, a, o, r, d, None, st))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        flib.check(L.fenv_rollout(env._h, T, a, o, r, d, None, st))
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for rnd in range(2):
    for kind in ("torch", "hipMalloc", "contiguous"):
        try:
            ptrs, keep = alloc(kind)
        except RuntimeError as ex:
            print(f"round {rnd} {kind:10s} {ex}", flush=True)
            continue
        torch.cuda.synchronize()
        hip.hipMemcpy(ctypes.c_void_p(ptrs[0]), ctypes.c_void_p(src.data_ptr()), sizes[0], 3)
        us = run(ptrs)
        print(f"round {rnd} {kind:10s} {us:7.1f} us per 10-step launch "
              f"({2.4642e9 / (us * 1e-6) / 8e12:.3f} of the HBM spec)", flush=True)
        if keep is None:
            for p in ptrs:
                hip.hipFree(ctypes.c_void_p(p))
        del keep
        torch.cuda.empty_cache()
