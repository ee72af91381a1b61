"""Host time of one config-3 MT19937 draw set (1,048,576 x 5 = 12.6M draws): fenv_host_reset_draws
into ordinary numpy memory (the library's 4-part parallel draw, no tags), best of 5, against the
env's own draw-ahead (the longest host call of a rollout window that holds reset events)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pkgload  # noqa: E402

pkg = pkgload.load()
from importlib import import_module  # noqa: E402

L = import_module(pkg.__name__ + "._lib")
F, N = 1 << 20, 5
out = {}
for F_ in (87000, F):
    px = np.zeros(F_ * N, np.float32)
    py = np.zeros(F_ * N, np.float32)
    gx = np.zeros(F_, np.float32)
    gy = np.zeros(F_, np.float32)
    best = 1e9
    for _ in range(5):
        t = time.perf_counter()
        L.check(L.lib().fenv_host_reset_draws(1, 0, F_, 0, F_, N,
                                              *(L.ptr(v) for v in (px, py, gx, gy))))
        best = min(best, time.perf_counter() - t)
    out[F_] = {"ms": best * 1e3, "ns_per_draw": best * 1e9 / (F_ * (2 * N + 2))}
print(json.dumps(out))
