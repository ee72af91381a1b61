"""Where do the non-kernel microseconds of bench.py's timed region go?  

Two 10-step fused rollouts of F formations x 5 agents (the driver's --steps 20 window), issued
through the C ABI exactly like bench.py, timed R times per variant; for every variant the
median wall time, the median event-timed kernel time and their difference (the fixed cost).

  bare_devsync   t0; launch; launch; torch.cuda.synchronize()            (the floor)
  bare_evsync    t0; launch; launch; event.record(); event.synchronize()
  ev_fresh       bare_devsync + fresh torch.cuda.Event()s recorded at the launch boundaries
                 (torch creates the HIP event lazily at its first record: inside the window)
  ev_pre         the same with events created and recorded once before the window
  waitstream     ev_pre + side.wait_stream(main) / main.wait_stream(side) (each creates and
                 records a fresh event) around a side-stream stats reduction of launch 1
  waitevent      the same dependencies through pre-created events (wait_event)
  waitevent_late waitevent with launch 2 issued before launch 1's side-stream stats work
  ev_start_only / ev_end_only / ev_both: bare_devsync with a timing event before the first
                 launch, after the last, or both (what each end's event costs)
  bench_*        bench.py's region (timing events at the ends only), ended by a device
                 synchronize, by polling the last event first, or by synchronizing on it first

    python tools/timed_region_probe.py [F ...]        (default 131072 1048576)
"""
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
dev = torch.device("cuda", 0)
T, N, R = 10, 5, int(os.environ.get("PROBE_REPS", 40))
vp = ctypes.c_void_p


def probe(F):
    env = venv.FormationEnv({"num_formation": F, "num_agents_per_formation": N,
                             "goal_in_obs": True}, log=False, device=dev, seed=0,
                            reset_mode="philox")
    A = env.num_envs
    acts = torch.rand((T, A, 2), device=dev) * 2 - 1
    obs = torch.empty((T, A, 8), device=dev)
    rew = torch.empty((T, A), device=dev)
    done = torch.empty((T, A), dtype=torch.bool, device=dev)
    part = torch.zeros((env.partial_count(), 2), device=dev)
    red = torch.zeros(2, dtype=torch.float64, device=dev)
    env.reset_tensor()
    main = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev)
    L = flib.lib()
    args = (env._h, T, vp(acts.data_ptr()), vp(obs.data_ptr()), vp(rew.data_ptr()),
            vp(done.data_ptr()))
    sp = vp(main.cuda_stream)
    ssp = vp(side.cuda_stream)
    pp, rp = vp(part.data_ptr()), vp(red.data_ptr())
    npart = env.partial_count()

    def launch(stat=False):
        L.fenv_rollout(*args, pp if stat else None, sp)

    def reduce_side():
        L.fenv_reduce_partials(pp, npart, rp, ssp)

    pre = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    dep = [torch.cuda.Event() for _ in range(2)]
    for e in pre + dep:
        e.record(main)
    fin = torch.cuda.Event()
    fin.record(main)
    torch.cuda.synchronize()

    def bare_devsync():
        t0 = time.perf_counter()
        launch()
        launch()
        torch.cuda.synchronize()
        return time.perf_counter() - t0, None

    def bare_evsync():
        t0 = time.perf_counter()
        launch()
        launch()
        fin.record(main)
        fin.synchronize()
        return time.perf_counter() - t0, None

    def ev_fresh():
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        t0 = time.perf_counter()
        ev[0].record(main)
        launch()
        ev[1].record(main)
        launch()
        ev[2].record(main)
        torch.cuda.synchronize()
        return time.perf_counter() - t0, ev[0].elapsed_time(ev[2])

    def ev_pre():
        t0 = time.perf_counter()
        pre[0].record(main)
        launch()
        pre[1].record(main)
        launch()
        pre[2].record(main)
        torch.cuda.synchronize()
        return time.perf_counter() - t0, pre[0].elapsed_time(pre[2])

    def waitstream():
        t0 = time.perf_counter()
        pre[0].record(main)
        launch(True)
        pre[1].record(main)
        side.wait_stream(main)
        reduce_side()
        launch()
        pre[2].record(main)
        main.wait_stream(side)
        torch.cuda.synchronize()
        return time.perf_counter() - t0, pre[0].elapsed_time(pre[2])

    def waitevent():
        t0 = time.perf_counter()
        pre[0].record(main)
        launch(True)
        pre[1].record(main)
        dep[0].record(main)
        side.wait_event(dep[0])
        reduce_side()
        dep[1].record(side)
        launch()
        pre[2].record(main)
        main.wait_event(dep[1])
        torch.cuda.synchronize()
        return time.perf_counter() - t0, pre[0].elapsed_time(pre[2])

    def waitevent_late():
        t0 = time.perf_counter()
        pre[0].record(main)
        launch(True)
        pre[1].record(main)
        dep[0].record(main)
        launch()
        pre[2].record(main)
        side.wait_event(dep[0])
        reduce_side()
        dep[1].record(side)
        main.wait_event(dep[1])
        fin.record(main)
        fin.synchronize()
        return time.perf_counter() - t0, pre[0].elapsed_time(pre[2])

    def bench_like(end):
        """bench.py's region at HEAD: start event, stats launch, plain mark, launch, end event,
        side-stream reduction issued after the second launch, main waits for it, fin; then the
        end of the window by `end`: devsync, poll (fin.query() loop, then devsync), evsync
        (fin.synchronize(), then devsync)."""
        def f():
            t0 = time.perf_counter()
            pre[0].record(main)
            launch(True)
            dep[0].record(main)
            launch()
            pre[2].record(main)
            side.wait_event(dep[0])
            reduce_side()
            dep[1].record(side)
            main.wait_event(dep[1])
            fin.record(main)
            if end == "poll":
                while not fin.query():
                    pass
            elif end == "evsync":
                fin.synchronize()
            torch.cuda.synchronize()
            return time.perf_counter() - t0, pre[0].elapsed_time(pre[2])
        return f

    def ev_start_only():
        t0 = time.perf_counter()
        pre[0].record(main)
        launch()
        launch()
        torch.cuda.synchronize()
        return time.perf_counter() - t0, None

    def ev_end_only():
        t0 = time.perf_counter()
        launch()
        launch()
        pre[2].record(main)
        torch.cuda.synchronize()
        return time.perf_counter() - t0, None

    def ev_both():
        t0 = time.perf_counter()
        pre[0].record(main)
        launch()
        launch()
        pre[2].record(main)
        torch.cuda.synchronize()
        return time.perf_counter() - t0, pre[0].elapsed_time(pre[2])

    variants = dict(ev_start_only=ev_start_only, ev_end_only=ev_end_only, ev_both=ev_both,
                    bare_devsync=bare_devsync, bare_evsync=bare_evsync, ev_fresh=ev_fresh,
                    ev_pre=ev_pre, waitstream=waitstream, waitevent=waitevent,
                    waitevent_late=waitevent_late, bench_devsync=bench_like("devsync"),
                    bench_poll=bench_like("poll"), bench_evsync=bench_like("evsync"))
    if os.environ.get("PROBE_ONLY"):
        variants = {k: v for k, v in variants.items() if k in os.environ["PROBE_ONLY"].split(",")}
    # device time of two launches, for the variants without events
    kern = []
    for _ in range(R):
        pre[0].record(main)
        launch()
        launch()
        pre[2].record(main)
        torch.cuda.synchronize()
        kern.append(pre[0].elapsed_time(pre[2]))
    res = {}
    for rnd in range(2):  # interleaved rounds: box drift hits every variant alike
        for name, fn in variants.items():
            for _ in range(5):  # warm (clock, first use of anything)
                fn()
            for _ in range(R // 2):
                w, k = fn()
                res.setdefault(name, []).append((w * 1e3, k))
    kmed = statistics.median(kern)
    out = {"formations": F, "agents": A, "launches": 2, "T": T, "reps": R,
           "kernel_ms_2launch_median": kmed}
    for name, v in res.items():
        wall = statistics.median(w for w, _ in v)
        ks = [k for _, k in v if k is not None]
        km = statistics.median(ks) if ks else kmed
        out[name] = {"wall_ms": wall, "kernel_ms": km, "fixed_us": (wall - km) * 1e3,
                     "wall_min_ms": min(w for w, _ in v)}
    env.release()
    return out


if __name__ == "__main__":
    sizes = [int(x) for x in sys.argv[1:]] or [131072, 1048576]
    for F in sizes:
        print(json.dumps(probe(F)), flush=True)
