"""Host scheduling jitter on the GPU box: gaps between consecutive time.perf_counter() reads in
a 2 s pure-Python loop (no GPU work), then the same while the process holds an idle HIP context
(torch initialised on cuda:0).  Reports gap counts over 20 / 50 / 100 us and the largest gaps.
    python tools/host_jitter_probe.py   -> one JSON line per phase
"""
import json
import time


def loop(label, seconds=2.0):
    pc = time.perf_counter
    t_end = pc() + seconds
    prev = pc()
    gaps = []
    n = 0
    while True:
        t = pc()
        d = t - prev
        if d > 20e-6:
            gaps.append(d)
        prev = t
        n += 1
        if t > t_end:
            break
    gaps.sort()
    print(json.dumps({"phase": label, "reads": n, "over_20us": len(gaps),
                      "over_50us": sum(1 for g in gaps if g > 50e-6),
                      "over_100us": sum(1 for g in gaps if g > 100e-6),
                      "largest_us": [round(g * 1e6, 1) for g in gaps[-8:]]}), flush=True)


loop("pure_python")
import torch  # noqa: E402
x = torch.zeros(1, device="cuda:0")
torch.cuda.synchronize()
loop("with_hip_context")
