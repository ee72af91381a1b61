#!/usr/bin/env python3
"""Headline benchmark: synthetic random-action rollouts of the formation env on MI355X.

Metric (BASELINE.json): agent-steps/sec (whole node) at 5 agents/formation, and the step
kernel's fraction of the HBM roofline.  Workload: BASELINE config 3 -- 1,048,576 formations x 5
agents (5,242,880 agents).  Formations are independent, so the ranks own disjoint contiguous
formation shards of one global env with no data-path collective.  With N > 1 GPUs the headline
is config 3 as written -- the 1M formations split over the ranks (strong scaling, `"scaling":
"strong"`) -- and the same line nests the weak-scaling measurement (1M formations on every rank,
`weak_scaling_line`); `--scaling weak` swaps the two, `--no-weak-line` skips the nested one.
A "step" is one env step of every agent; steps run as fused rollouts of
`--chunk` steps per launch (SB3's n_steps=10 rollout, vectorized_env.py:128) writing obs /
reward / done for every step into a device rollout buffer, with the actions read from HBM
(inputs resident before the timed region).  Episode stats are reduced on device and all-reduced
over RCCL every --stats-every rollouts on a side stream.

Secondary lines (N = 1, after the timed region): the fused policy rollout (config 2), the PPO
update, MT19937 reset mode, the random-action launch, the numpy (PCIe-inclusive) face, configs
1 and 4, the single-step face, and the CPU baseline.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "agent-steps/sec (whole node) at 5 agents/formation; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)


def rollout_bytes_per_launch(A: int, N: int, D: int, T: int) -> float:
    """Algorithmic HBM bytes of one fenv_rollout launch:
    per agent-step: action 8 + obs 4D + reward 4 + done 1; per agent-launch: position read +
    write 16, formation goal 8 + steps_since_reset 4+4 + episode 4 read, per formation."""
    per_step = 8 + 4 * D + 4 + 1
    per_launch = 16 + (8 + 8 + 4) / N
    return A * (T * per_step + per_launch)


def _cpu_oracle_rate(F: int, N: int, D: int, threads: int, budget_s: float):
    """Step `threads` independent shards of F formations (one C oracle env per thread, ctypes
    drops the GIL for the call) until `budget_s` has passed; returns (agent-steps/s, steps)."""
    import threading
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import COracleEnv
    shards = [F // threads + (1 if t < F % threads else 0) for t in range(threads)]
    envs = [COracleEnv(f, N, D == 8, t) for t, f in enumerate(shards)]
    for e in envs:
        e.reset()
    acts = [[np.random.default_rng(t * 4 + k).uniform(-1, 1, (f * N, 2)).astype(np.float32)
             for k in range(4)] for t, f in enumerate(shards)]
    steps = [0] * threads
    t0 = time.perf_counter()
    deadline = t0 + budget_s

    def run(t):
        e, a, k = envs[t], acts[t], 0
        while time.perf_counter() < deadline:
            e.step_inplace(a[k % 4])
            k += 1
        steps[t] = k

    ths = [threading.Thread(target=run, args=(t,)) for t in range(threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    el = time.perf_counter() - t0
    return sum(f * N * k for f, k in zip(shards, steps)) / el, min(steps), el


# The reference CPU env itself, measured in the build container:
# it cannot travel to the GPU box, so it is carried as a labelled constant, never re-run here.
REFERENCE_CPU_MEASURED = {
    "value_range": [6.2e3, 1.0e4], "unit": "agent-steps/s",
    "config": "config0: 1000 formations x 5 agents (cfg/config.yaml defaults)", "threads": 1,
    "host": "8 vCPU Xeon (KVM), build container", "kind": "reference",
    "source": "SURVEY.md §6 / BASELINE.md (measured by importing /root/reference; not re-run)"}


def cpu_share() -> tuple[int, str]:
    """Host threads this job may run at once: the affinity mask, capped by the cgroup CPU quota
    (cpu.max `quota period`).  On the GPU box the affinity shows all 256 CPUs and the quota is
    1600000 / 100000 = 16 CPUs; the C port's rate there peaks at 16 threads (4.5e8) and falls
    beyond (24: 4.4e8, 32: 4.2e8, 64: 2.0e8 -- throttled; tools/cpu_share_probe.py,
    profiles/r5_cpu_share.json).  Returns (threads, how they were found)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    for p in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            parts = open(p).read().split()
        except OSError:
            continue
        if p.endswith("cpu.max") and len(parts) == 2 and parts[0] != "max":
            quota = int(parts[0]) / int(parts[1])
        elif p.endswith("cfs_quota_us") and parts and int(parts[0]) > 0:
            period = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            quota = int(parts[0]) / period
        break
    if quota is None:
        return max(1, aff), f"affinity {aff}, no cgroup CPU quota"
    return max(1, min(aff, int(quota))), f"affinity {aff}, cgroup CPU quota {quota:g}"


def cpu_baseline(N: int, D: int, budget_s: float) -> dict:
    """Time the bit-exact C port of the reference env (oracle/fenv_oracle.c) on bounded samples:
    BASELINE config 0 (1000 x 5, the reference's default CPU run) and config 1 (4096 x 5) on one
    thread, then a sample of the headline workload (65,536 x 5 formations, one thread, then one
    thread per CPU of this job's share (cpu_share: 16 on the GPU box), over formation shards).
    `value` is the multi-threaded rate on the headline sample; `cores` the threads it used."""
    F = 65536
    threads, share = cpu_share()
    small = budget_s / 6
    configs = {}
    for name, (fc, nc) in (("config0", (1000, 5)), ("config1", (4096, 5))):
        r, k, el = _cpu_oracle_rate(fc, nc, D, 1, small)
        configs[name] = {"value": r, "unit": "agent-steps/s", "cores": 1, "kind": "port",
                         "sample": f"{fc} formations x {nc} agents, {k} env steps ({el:.1f} s), "
                                   f"1 thread"}
    one, one_steps, one_el = _cpu_oracle_rate(F, N, D, 1, budget_s / 3)
    many, many_steps, many_el = _cpu_oracle_rate(F, N, D, threads, budget_s / 3)
    return {"value": many, "unit": "agent-steps/s", "cores": threads, "kind": "port",
            "single_thread_value": one,
            "sample": f"{F} formations x {N} agents: 1 thread {one_steps} env steps "
                      f"({one_el:.1f} s), then {threads} threads over {threads} formation "
                      f"shards >= {many_steps} env steps each ({many_el:.1f} s); "
                      f"oracle/fenv_oracle.c (bit-exact C port of simulate.py/"
                      f"vectorized_env.py); host reports {os.cpu_count()} CPUs; "
                      f"threads = this job's CPU share ({share})",
            "configs": configs,
            "reference_measured": REFERENCE_CPU_MEASURED}


def _warm(fn, min_ms: float = 300.0) -> int:
    """Run `fn` back to back for at least `min_ms` of wall time, then synchronize: each
    secondary line starts from the clocks a sustained load holds (a few warm-up calls after an
    idle gap left the fused policy rollout ~15 % slow, tools/collect_overhead.py).  Returns the
    number of calls."""
    import torch
    n, t0 = 0, time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < min_ms or n < 3:
        fn()
        n += 1
        if n % 64 == 0:
            torch.cuda.synchronize()  # bounds the queue (short kernels issue faster than they run)
    torch.cuda.synchronize()
    return n


def policy_rollout_bench(pkgname: str, dev, formations: int, agents: int, rollouts: int) -> dict:
    """Secondary measurement (BASELINE config 2): on-device PPO rollout collection with the MFMA
    policy forward + env step per step (65536 formations x 10 agents), plus the policy
    kernel's fp32-MFMA utilisation."""
    import torch
    from importlib import import_module
    venv = import_module(pkgname + ".vectorized_env")
    pol_mod = import_module(pkgname + ".policy")
    ro = import_module(pkgname + ".rollout")
    cfg = {"num_formation": formations, "num_agents_per_formation": agents, "goal_in_obs": True}
    env = venv.FormationEnv(cfg, log=False, device=dev, seed=1, reset_mode="philox")
    A = env.num_envs
    pol = pol_mod.MlpPolicy(8, device=dev, seed=0)
    buf = ro.RolloutBuffer(10, A, 8, dev)
    col = ro.RolloutCollector(env, pol, buf, seed=0)
    _warm(col.collect)
    t0 = time.perf_counter()
    for _ in range(rollouts):
        col.collect()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    # the fused collection kernel alone (no GAE launch), HIP events on its stream
    bufs = dict(obs=buf.observations, mu=buf.mu, action=buf.actions, clipped=buf.clipped,
                value=buf.values, log_prob=buf.log_probs, reward=buf.rewards,
                episode_start=buf.episode_starts, done=buf.dones,
                last_done=col.last_episode_starts, last_obs=col.last_obs,
                last_value=col._last_values)
    ka, kb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    _warm(lambda: env.policy_rollout(pol.flat, 10, bufs, seed=0, offset=500), 100.0)
    ka.record()
    for r in range(rollouts):
        env.policy_rollout(pol.flat, 10, bufs, seed=0, offset=1000 + 10 * r)
    kb.record()
    torch.cuda.synchronize()
    pr_ms = ka.elapsed_time(kb) / rollouts
    # policy kernel alone, HIP events on its stream
    obs = buf.observations[0]
    out = dict(mu=buf.mu[0], value=buf.values[0], action=buf.actions[0],
               log_prob=buf.log_probs[0], clipped=buf.clipped[0])
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(20)]
    _warm(lambda: pol.forward(obs, out=out, seed=0, offset=0), 100.0)
    for a, b in evs:
        a.record()
        pol.forward(obs, out=out, seed=0, offset=0)
        b.record()
    torch.cuda.synchronize()
    pk_ms = sum(a.elapsed_time(b) for a, b in evs) / len(evs)
    flop = 18816.0 * A           # fp32-equivalent FLOP of one policy_forward over the batch
    f16 = 57344.0 * A            # split-f16 MFMA FLOP actually issued (56 MFMAs per 32 agents)
    return {"workload": f"config2: {formations} formations x {agents} agents, PPO rollout "
                        f"(n_steps=10): fused MFMA policy forward + env step per step, GAE",
            "value": A * 10 * rollouts / el, "unit": "agent-steps/s",
            "rollout_kernel_ms": pr_ms,
            "roofline": policy_rollout_roofline(pr_ms),
            "policy_kernel_ms": pk_ms,
            "policy_fp32_equiv_tflops": flop / (pk_ms * 1e-3) / 1e12,
            "policy_f16_mfma_tflops": f16 / (pk_ms * 1e-3) / 1e12,
            "f16_mfma_dense_peak_tflops": 2516.6,
            "f16_mfma_frac": f16 / (pk_ms * 1e-3) / 1e12 / 2516.6,
            "arithmetic": "split-f16 MFMA (hi*hi + hi*lo + lo*hi, fp32 accumulate), fp32 tanh/heads",
            "bound": "VALU issue (256 exp+rcp tanh per agent-step), see DESIGN.md"}


SIMDS, SCLK_HZ = 1024, 2.4e9  # MI355X: 256 CUs x 4 SIMDs, 2.4 GHz peak engine clock


def policy_rollout_roofline(kernel_ms: float):
    """Roofline of the fused policy rollout (k_policy_rollout): it is bound by VALU issue, not by
    HBM (~78 B per agent-step) or the MFMA pipe.  achieved = the kernel's VALU-active SIMD-cycles
    per launch (SQ_ACTIVE_INST_VALU x 4, PMC, profiles/r4_policy_pmc_sq.json) / the launch time
    measured live in this run; peak = every SIMD's VALU busy every cycle (1024 x 2.4 GHz).
    mfma_busy_frac the same way from SQ_VALU_MFMA_BUSY_CYCLES."""
    # the PMC passes of the current round (tools/policy_pmc.sh at HEAD), else an older round's
    src = next((f for f in ("r4_policy_pmc_sq.json", "r2_policy_pmc_sq.json")
                if os.path.exists(os.path.join(ROOT, "profiles", f))), None)
    if src is None:
        return None
    p = os.path.join(ROOT, "profiles", src)
    ks = json.load(open(p)).get("kernels", {})
    k = next((v for n, v in ks.items() if "k_policy_rollout" in n), None)
    if not k or "SQ_ACTIVE_INST_VALU" not in k:
        return None
    peak = SIMDS * SCLK_HZ
    valu = 4.0 * k["SQ_ACTIVE_INST_VALU"] / (kernel_ms * 1e-3)
    out = {"bound": "valu-issue", "achieved": valu, "peak": peak,
           "unit": "VALU-active SIMD-cycles/s", "frac": valu / peak,
           "valu_insts_per_launch": k.get("SQ_INSTS_VALU"),
           "kernel": "k_policy_rollout (fenv_policy_rollout)", "kernel_ms": kernel_ms,
           "pmc_source": f"profiles/{src}"}
    if "SQ_VALU_MFMA_BUSY_CYCLES" in k:
        out["mfma_busy_frac"] = k["SQ_VALU_MFMA_BUSY_CYCLES"] / (kernel_ms * 1e-3) / peak
    if "SQ_WAVE_CYCLES" in k:
        out["avg_waves_per_simd"] = 4.0 * k["SQ_WAVE_CYCLES"] / (kernel_ms * 1e-3) / peak
    if "GRBM_GUI_ACTIVE" in k and "SQ_ACTIVE_INST_ANY" in k:
        # within the profiled run itself: the share of the clocked SIMD-cycles (GRBM_GUI_ACTIVE is
        # summed over the 8 XCDs) in which the SIMD issued any instruction (VALU, MFMA, LDS,
        # SALU, branch) -- how close the kernel is to the issue limit, whatever the clock
        clocked = k["GRBM_GUI_ACTIVE"] / 8.0 * SIMDS
        out["issue_busy_frac_clocked"] = 4.0 * k["SQ_ACTIVE_INST_ANY"] / clocked
        out["valu_busy_frac_clocked"] = 4.0 * k["SQ_ACTIVE_INST_VALU"] / clocked
    return out


def env_config_bench(pkgname: str, dev, formations: int, agents: int, launches: int = 50,
                     T: int = 10) -> dict:
    """Secondary env-only lines (BASELINE.json configs[1] and [4]): fused T-step rollouts of the given
    shape with HBM-resident actions, avg launch time from HIP events on the launch stream."""
    import torch
    from importlib import import_module
    venv = import_module(pkgname + ".vectorized_env")
    cfg = {"num_formation": formations, "num_agents_per_formation": agents, "goal_in_obs": True}
    env = venv.FormationEnv(cfg, log=False, device=dev, seed=0, reset_mode="philox")
    A = env.num_envs
    acts = torch.rand((T, A, 2), device=dev) * 2 - 1
    obs = torch.empty((T, A, 8), device=dev)
    rew = torch.empty((T, A), device=dev)
    done = torch.empty((T, A), dtype=torch.bool, device=dev)
    env.reset_tensor()
    _warm(lambda: env.rollout(acts, obs, rew, done), 200.0)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    a.record()
    for _ in range(launches):
        env.rollout(acts, obs, rew, done)
    b.record()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    eager_ms = a.elapsed_time(b) / launches
    # Device time per launch without the Python issue cost: the same launches captured in a HIP
    # graph and replayed (a small grid's launch is shorter than the ~10-20 us it takes the host
    # to issue one through the Python face, so back-to-back eager launches measure the host)
    ms, timing = eager_ms, "HIP events around back-to-back eager launches"
    try:
        K = max(1, min(launches, 100))
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(K):
                env.rollout(acts, obs, rew, done)
        _warm(g.replay, 100.0)
        reps = max(1, launches // K)
        a.record()
        for _ in range(reps):
            g.replay()
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / (reps * K)
        timing = f"HIP events around {reps} replays of a HIP graph of {K} launches"
    except Exception as ex:  # capture unsupported here: keep the eager figure
        timing += f" (graph capture failed: {type(ex).__name__})"
    byts = rollout_bytes_per_launch(A, agents, 8, T)
    shape = (f"fused {T}-step rollouts" if T > 1 else
             "one env step per launch (fenv_step: state read + write every step)")
    return {"workload": f"{formations} formations x {agents} agents, {shape}",
            "value": A * T * launches / el, "unit": "agent-steps/s", "avg_kernel_ms": ms,
            "eager_launch_ms": eager_ms, "timing": timing,
            "algorithmic_bytes_per_launch": byts,
            "hbm_gbs": byts / (ms * 1e-3) / 1e9, "hbm_frac": byts / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS}


def random_action_bench(pkgname: str, dev, formations: int, agents: int, launches: int = 200,
                        T: int = 10) -> dict:
    """Secondary line: the north star's "synthetic random-action rollouts" with the actions drawn
    inside the kernel (fenv_rollout_random, Philox) instead of read from HBM -- same env work,
    8 B/agent-step less traffic.  Algorithmic bytes exclude the action read."""
    import torch
    from importlib import import_module
    venv = import_module(pkgname + ".vectorized_env")
    cfg = {"num_formation": formations, "num_agents_per_formation": agents, "goal_in_obs": True}
    env = venv.FormationEnv(cfg, log=False, device=dev, seed=0, reset_mode="philox")
    A = env.num_envs
    obs = torch.empty((T, A, 8), device=dev)
    rew = torch.empty((T, A), device=dev)
    done = torch.empty((T, A), dtype=torch.bool, device=dev)
    env.reset_tensor()
    _warm(lambda: env.rollout_random(T, 7, 0, obs, rew, done), 200.0)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    a.record()
    for k in range(launches):
        env.rollout_random(T, 7, (k + 3) * T, obs, rew, done)
    b.record()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ms = a.elapsed_time(b) / launches
    byts = rollout_bytes_per_launch(A, agents, 8, T) - 8.0 * A * T
    return {"workload": f"{formations} formations x {agents} agents, fused {T}-step rollouts, "
                        f"in-kernel Philox U(-1,1) actions",
            "value": A * T * launches / el, "unit": "agent-steps/s", "avg_kernel_ms": ms,
            "algorithmic_bytes_per_launch": byts,
            "hbm_gbs": byts / (ms * 1e-3) / 1e9, "hbm_frac": byts / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS}


def numpy_face_bench(pkgname: str, dev, formations: int, agents: int, steps: int) -> dict:
    """The PCIe-inclusive rate: the reference's own interface, ``FormationEnv.step(np.ndarray)``
    (vectorized_env.py:68-82, what SB3's VecEnv loop calls): the kernel reads the actions from
    and writes obs / reward / done to device-mapped host memory, so every step crosses PCIe.
    Never the headline `value` (its inputs are not HBM-resident)."""
    import numpy as np
    from importlib import import_module
    venv = import_module(pkgname + ".vectorized_env")
    cfg = {"num_formation": formations, "num_agents_per_formation": agents, "goal_in_obs": True}
    env = venv.FormationEnv(cfg, log=False, device=dev, seed=0, reset_mode="philox")
    A = env.num_envs
    rng = np.random.default_rng(7)
    acts = [rng.uniform(-1, 1, (A, 2)).astype(np.float32) for _ in range(2)]
    env.reset()
    for k in range(3):
        env.step(acts[k % 2])
    t0 = time.perf_counter()
    for k in range(steps):
        env.step(acts[k % 2])
    el = time.perf_counter() - t0
    env.release()
    pcie_b = A * (2 * 4 + 8 * 4 + 4 + 1)  # actions in; obs, reward, done out
    return {"workload": f"{formations} formations x {agents} agents, FormationEnv.step(numpy) "
                        f"x {steps}", "value": A * steps / el, "unit": "agent-steps/s",
            "ms_per_step": 1e3 * el / steps, "pcie_bytes_per_step": pcie_b,
            "pcie_gbs": pcie_b * steps / el / 1e9}


def mt_mode_bench(pkgname: str, dev, formations: int, agents: int, steps: int = 2100,
                  T: int = 10) -> dict:
    """The same fused rollouts in MT19937 reset mode (the reference's exact RNG stream: every
    reset set replayed on the host and staged), over a window holding two reset
    events (episode = 1,002 steps), with the Philox rate of the same window beside it."""
    import torch
    from importlib import import_module
    venv = import_module(pkgname + ".vectorized_env")
    out = {"workload": f"{formations} formations x {agents} agents, fused {T}-step rollouts, "
                       f"{steps} steps (two reset events), aligned episodes", "unit": "agent-steps/s"}
    for mode in ("mt19937", "philox"):
        cfg = {"num_formation": formations, "num_agents_per_formation": agents, "goal_in_obs": True}
        env = venv.FormationEnv(cfg, log=False, device=dev, seed=0, reset_mode=mode)
        A = env.num_envs
        acts = torch.rand((T, A, 2), device=dev) * 2 - 1
        obs = torch.empty((T, A, 8), device=dev)
        rew = torch.empty((T, A), device=dev)
        done = torch.empty((T, A), dtype=torch.bool, device=dev)
        env.reset_tensor()
        for _ in range(3):
            env.rollout(acts, obs, rew, done)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        k = 0
        while k < steps:
            L = min(T, steps - k)
            env.rollout(acts[:L], obs[:L], rew[:L], done[:L])
            k += L
        torch.cuda.synchronize()
        out[mode] = A * steps / (time.perf_counter() - t0)
        env.release()
        del env, acts, obs, rew, done
        torch.cuda.empty_cache()
    out["value"] = out["mt19937"]
    out["mt19937_over_philox"] = out["mt19937"] / out["philox"]
    return out


def secondary(fn, *a):
    """A secondary line (after the timed region): an error in it is reported in its own field
    instead of taking the headline line down with it."""
    try:
        return fn(*a)
    except Exception as ex:
        return {"error": f"{type(ex).__name__}: {ex}"}


def ppo_update_bench(pkgname: str, dev, formations: int = 1000, agents: int = 5,
                     updates: int = 2) -> dict:
    """Secondary measurement: SB3's PPO.train at the reference's training config
    (vectorized_env.py:126-131: n_steps 10, batch 64, 10 epochs over 1000 x 5 agents) with the
    fused ppo_update kernel; one update = 7,820 minibatch steps."""
    import torch
    from importlib import import_module
    venv = import_module(pkgname + ".vectorized_env")
    ppo_mod = import_module(pkgname + ".ppo")
    cfg = {"num_formation": formations, "num_agents_per_formation": agents, "goal_in_obs": True}
    env = venv.FormationEnv(cfg, log=False, device=dev, seed=0, reset_mode="philox")
    m = ppo_mod.PPO(env, ppo_mod.PPOConfig(), seed=0)
    with torch.no_grad():
        m.collector.collect()
    m.train()  # warm-up (allocates the Adam state)
    torch.cuda.synchronize()
    el, col = 0.0, 0.0
    for _ in range(updates):
        t0 = time.perf_counter()
        with torch.no_grad():
            m.collector.collect()
        torch.cuda.synchronize()
        col += time.perf_counter() - t0
        t0 = time.perf_counter()
        m.train()
        torch.cuda.synchronize()
        el += time.perf_counter() - t0
    n = env.num_envs * m.cfg.n_steps
    mb = m.cfg.n_epochs * -(-n // m.cfg.batch_size)
    per_mb = el / (updates * mb)
    flop = 56448.0 * m.cfg.batch_size  # ~3 x 18,816 FLOP per sample (forward + backward)
    return {"workload": f"PPO.train, {formations} x {agents} agents, n_steps 10, batch 64, "
                        f"10 epochs (SB3 defaults of the reference's PPO call)",
            "path": "fused" if m.use_fused else ("graph" if m.use_graph else "eager"),
            "ms_per_update": el / updates * 1e3, "us_per_minibatch": per_mb * 1e6,
            # one whole training iteration (model.learn's loop body): rollout collection (fused
            # policy + env kernel, GAE) + the update, in env agent-steps per second
            "collect_ms": col / updates * 1e3,
            "training_agent_steps_per_s": n / ((el + col) / updates),
            "samples_per_s": n * m.cfg.n_epochs / (el / updates),
            "gflops": flop / per_mb / 1e9,
            "exchange_reruns": m.exchange_retries,
            "mfma_pipe": ppo_pmc_mfma(),
            "note": "actor and critic on one CU each (a minibatch depends on the previous "
                    "one's parameters); one CU's fp32 peak is ~614 GFLOP/s"}


def ppo_pmc_mfma():
    """Counter-backed MFMA-pipe occupancy of k_ppo_update from the committed PMC passes
    (tools/ppo_pmc.sh -> profiles/r4_ppo_pmc_sq.json, else round 3's; not measured in this
    run).  The kernel runs 8 waves on 8 SIMDs (4 per CU, actor and critic CU);
    SQ_VALU_MFMA_BUSY_CYCLES counts cycles summed over the chip, GRBM_GUI_ACTIVE the kernel's
    cycles summed over the 8 XCDs."""
    p = os.path.join(ROOT, "profiles", "r4_ppo_pmc_sq.json")
    if not os.path.exists(p):
        p = os.path.join(ROOT, "profiles", "r3_ppo_pmc_sq.json")
    try:
        k = next(iter(json.load(open(p))["kernels"].values()))
        cycles = k["GRBM_GUI_ACTIVE"] / 8.0
        return {"busy_frac": k["SQ_VALU_MFMA_BUSY_CYCLES"] / 8.0 / cycles,
                "mfma_per_dispatch": k["SQ_INSTS_MFMA"], "kernel_cycles": cycles,
                "pmc_source": os.path.relpath(p, ROOT)}
    except Exception as ex:  # noqa: BLE001
        return {"error": f"{type(ex).__name__}: {ex}"}


def load_pmc_traffic(workload: str):
    """HBM bytes per launch measured by separate rocprofv3 PMC passes (tools/gpu_pmc.sh ->
    profiles/pmc_traffic.json).  Not measured in this run: returned with its source file."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None, None
    try:
        d = json.load(open(p))
        if d.get("workload") == workload:
            return d.get("hbm_bytes_per_launch"), "profiles/pmc_traffic.json"
    except Exception:
        pass
    return None, None


def hbm_ceiling(acts, obs, rew, done, A: int, T: int, D: int, stream, reps: int = 20):
    """Same-box HBM ceiling of the rollout's byte mix (tools/calib/hbm_ceiling.hip): the exact
    streams of one launch (45 B per agent-step at D = 8) with no arithmetic, every access a whole
    128-B-aligned float4 run, into this run's own rollout buffers, timed with HIP events on the
    launch stream.  Measured after the timed region, never inside it.  None when the library is
    not built or the shape does not apply (D != 8)."""
    import ctypes
    p = os.path.join(ROOT, "tools", "calib", "libhbm_ceiling.so")
    if D != 8 or not os.path.exists(p):
        return None
    lib = ctypes.CDLL(p)
    lib.hbm_ceiling_chunk.restype = ctypes.c_int
    lib.hbm_ceiling_mix_ms.restype = ctypes.c_double
    lib.hbm_ceiling_mix_ms.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int64, ctypes.c_int32,
                                                               ctypes.c_int32, ctypes.c_void_p]
    ch = lib.hbm_ceiling_chunk()
    Ac = A - A % ch
    if Ac <= 0:
        return None
    ms = lib.hbm_ceiling_mix_ms(acts.data_ptr(), obs.data_ptr(), rew.data_ptr(), done.data_ptr(),
                                Ac, T, reps, ctypes.c_void_p(stream.cuda_stream))
    if ms <= 0:
        return None
    byts = 45.0 * Ac * T
    return {"achieved": byts / (ms * 1e-3) / 1e9, "unit": "GB/s", "ms_per_launch": ms,
            "agents": Ac, "steps": T,
            "kernel": "k_mix (tools/calib/hbm_ceiling.hip): the launch's action read and obs / "
                      "reward / done writes, no arithmetic, whole aligned float4 runs; the "
                      "faster of plain and non-temporal stores"}


GATE_PREFIX = 64  # launches issued behind the launch gate before it is released (bench window)
ALIGN_MARGIN_NS = 1_000_000  # N > 1: the windows start this long after the ranks agree on when


class _Gate:
    """bench's launch gate: fenv_stream_gate on the launch stream over a word of device-mapped
    host memory (include/fenv.h).  arm() enqueues the gate wave (a new release value each time),
    release() stores the value from the host -- one plain memory write, no HIP call -- and
    status() reads what the wave recorded.  probe() measures the release latency: the host stores
    the value into an armed gate and spins until it sees the wave's status word, so one sample is
    host store -> the wave's poll sees it -> its status store -> the host's read sees that."""

    TIMEOUT_US = 5_000_000  # the wave exits after 5 s whatever the host does

    def __init__(self, flib, L, dev, stream):
        import ctypes
        import numpy as np
        self.L, self.flib = L, flib
        self.blk = flib.HostBlock(dev, [("flag", np.uint32, (16,)), ("status", np.uint32, (16,))])
        self.blk.flag[:] = 0
        self.stream = ctypes.c_void_p(stream.cuda_stream)
        self.value = 0
        if os.environ.get("FENV_BENCH_GATE_TEST") == "no-release":
            self.TIMEOUT_US = 20_000
        self.arm()      # first use (module load of the kernel) outside any window
        self.release()
        stream.synchronize()

    def arm(self):
        """Enqueue the gate wave (a new release value)."""
        self.value = (self.value + 1) & 0xFFFFFFFF or 1
        self.blk.status[:4] = 0
        rc = self.L.fenv_stream_gate(self.blk.dev("flag"), self.value, self.TIMEOUT_US,
                                     self.blk.dev("status"), self.stream)
        if rc:
            self.flib.check(rc, "fenv_stream_gate")

    def release(self):
        if os.environ.get("FENV_BENCH_GATE_TEST") == "no-release":  # test hook: let it time out
            return
        self.blk.flag[0] = self.value

    def status(self) -> dict:
        st = self.blk.status
        return {"released": int(st[0]), "polls": int(st[1]),
                "held_us": ((int(st[3]) << 32) | int(st[2])) / 1e3}

    def probe(self, reps: int = 21) -> dict:
        us = []
        for _ in range(reps):
            self.arm()
            t = time.perf_counter()
            while time.perf_counter() - t < 300e-6:  # the wave is polling by now
                pass
            t = time.perf_counter()
            self.release()
            while self.blk.status[0] == 0 and time.perf_counter() - t < 1.0:
                pass
            us.append((time.perf_counter() - t) * 1e6)
        import torch
        torch.cuda.synchronize()
        us.sort()
        return {"roundtrip_us_median": us[len(us) // 2], "roundtrip_us_max": us[-1],
                "reps": reps,
                "what": "host flag store -> gate wave sees it -> its status store reaches host "
                        "memory -> the spinning host sees it (two bus crossings)"}


def window_summary(w: dict, total_agents: int, steps: int) -> dict:
    """The JSON fields of one timed window (max over ranks)."""
    return {"value": total_agents * steps / w["elapsed_max"],
            "kernel_value": total_agents * steps / (w["kern_ms_max"] * 1e-3),
            "ms_per_step": w["elapsed_max"] * 1e3 / steps,
            "fixed_overhead_ms": w["elapsed_max"] * 1e3 - w["kern_ms_max"],
            "kernel_ms_timed": w["kern_ms_max"], "host_issue_ms": w["host_issue_ms"]}


def launch_plan(steps: int, T: int) -> list[int]:
    """Launch lengths covering exactly `steps` env steps in fused chunks of <= T steps."""
    full, rem = divmod(int(steps), int(T))
    return [T] * full + ([rem] if rem else [])


def stagger_episodes(env, pdist_first: int) -> None:
    """Spread the formations' episode phase (steps_since_reset) uniformly over the 1002-step
    episode (simulate.py:111,231), as a long training run reaches when episodes desynchronise:
    every timed window then contains the steady-state reset rate (1/1002 of the formations per
    step, drawn in-kernel by Philox) instead of none or all of them."""
    import torch
    px, py, gx, gy, t = env.get_state()
    F = t.numel()
    ep = env.max_steps + 2
    t = ((torch.arange(F, device=t.device, dtype=torch.int64) + pdist_first) % ep).to(torch.int32)
    env.set_state(px, py, gx, gy, t)


def run_config3(args, pkg, rank: int, world: int, dev, total_formations: int, scaling: str):
    """One headline measurement (BASELINE config 3 shape) over `total_formations` formations
    sharded contiguously over the ranks; returns the JSON line's fields on rank 0, None
    elsewhere.  Every rank builds its own shard env, buffers and streams; the env is released
    before returning so a second measurement starts from free HBM."""
    import torch
    from importlib import import_module
    venv = import_module(pkg.__name__ + ".vectorized_env")
    pdist = import_module(pkg.__name__ + ".distributed")
    N, T = args.agents, args.chunk
    D = 6 if args.no_goal else 8
    first, F = pdist.shard_range(total_formations, rank, world)
    cfg = {"num_formation": F, "num_agents_per_formation": N, "goal_in_obs": not args.no_goal}
    env = venv.FormationEnv(cfg, log=False, device=dev, seed=0, reset_mode=args.reset_mode,
                            first_formation=first, total_formations=total_formations)
    A = F * N
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    acts = [(torch.rand((T, A, 2), device=dev, generator=g) * 2 - 1) for _ in range(2)]
    obs = torch.empty((T, A, D), dtype=torch.float32, device=dev)
    rew = torch.empty((T, A), dtype=torch.float32, device=dev)
    done = torch.empty((T, A), dtype=torch.bool, device=dev)
    # Stats pipeline: a stats launch writes its per-wave {reward, done} records into partials[s]
    # on the main stream and records mark[s]; once the NEXT launch has been issued, the side
    # stream waits for mark[s], reduces partials[s] (deterministic order) into reds[s] and
    # all-reduces the two doubles over RCCL, overlapped with that launch; the stats launch that
    # next reuses slot s first waits for the reducer's event of that slot.  Every event the
    # region records is created and recorded once before it (torch creates a HIP event lazily at
    # its first record, and Stream.wait_stream creates a fresh one per call), and every library
    # call in it goes straight through the C ABI with pre-built arguments.
    partials = [torch.zeros((env.partial_count(), 2), dtype=torch.float32, device=dev)
                for _ in range(2)]
    reds = [torch.zeros(2, dtype=torch.float64, device=dev) for _ in range(2)]
    main_s = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev)
    stats = pdist.StatsReducer(2, dev, stream=side)
    mark = [torch.cuda.Event() for _ in range(2)]
    freed = [None, None]  # the reducer event after which partials[s] may be rewritten
    env.reset_tensor()
    phase = args.episode_phase if args.reset_mode == "philox" else "aligned"
    if phase == "staggered":
        stagger_episodes(env, first)
    nstat = [0]
    pending = []  # (launch index, slot) of stats launches whose reduction is not issued yet

    # Full-length launches go straight through the C ABI (include/fenv.h fenv_rollout,
    # fenv_reduce_partials) with pre-built arguments: the Python face's per-call validation
    # (~10-20 us of host time) would sit in front of the timed region's first launch.  The
    # buffers are validated once, here, by calls through the Python face.
    import ctypes
    flib = import_module(pkg.__name__ + "._lib")
    L_abi = flib.lib()
    vp = ctypes.c_void_p
    abi_stream = vp(main_s.cuda_stream)
    abi_args = [(env._h, T, vp(acts[k].data_ptr()), vp(obs.data_ptr()), vp(rew.data_ptr()),
                 vp(done.data_ptr())) for k in range(2)]
    abi_part = [vp(p.data_ptr()) for p in partials]
    npart = env.partial_count()
    abi_red = {(k, st): (abi_part[k], npart, vp(reds[k].data_ptr()), vp(st.cuda_stream))
               for k in range(2) for st in (main_s, side)}
    env.rollout(acts[0], obs, rew, done, partial=partials[0])
    env.reduce_partials(partials[0], reds[0])
    for e in mark:
        e.record(main_s)

    def issue_stats(s, st):
        """Reduce partials[s] into reds[s] and all-reduce it, on stream `st` (after mark[s])."""
        if st is not main_s:
            st.wait_event(mark[s])
        rc = L_abi.fenv_reduce_partials(*abi_red[(s, st)])
        if rc:
            flib.check(rc, "fenv_reduce_partials")
        stats.submit(reds[s], stream=st)
        freed[s] = stats.ready()

    def flush(before=None, last=False):
        """Issue the reductions of the pending stats launches (those before launch index
        `before`; all if None).  A reduction with no launch left to hide under (`last`) runs on
        the main stream: no cross-stream hop before the closing synchronize."""
        while pending and (before is None or pending[0][0] < before):
            _, s = pending.pop(0)
            issue_stats(s, main_s if last else side)

    stall_us = float(os.environ.get("FENV_BENCH_STALL_US", "0") or 0)

    def launch(k, L, stat=False, ev=None):
        """Launch k of a region: one fused rollout of L steps (actions of slot nstat-parity;
        stats if `stat`).  `ev` is recorded on the launch stream right before the kernel (after
        any stream-ordering call)."""
        s = nstat[0] % 2
        if stall_us and k == 1:
            # test hook (FENV_BENCH_STALL_US): a host stall of this length right before the
            # window's second launch is issued, like the 80-250 us ones round 5 saw in HIP calls
            t = time.perf_counter()
            while (time.perf_counter() - t) * 1e6 < stall_us:
                pass
        if stat and freed[s] is not None and not freed[s].query():
            # (a reduction the host already saw complete needs no wait packet in the queue)
            main_s.wait_event(freed[s])
        stamp("stats wait")
        if ev is not None:
            ev.record(main_s)
            stamp("start event")
        if L == T:
            rc = L_abi.fenv_rollout(*abi_args[s], abi_part[s] if stat else None, abi_stream)
            if rc:
                flib.check(rc, "fenv_rollout")
        else:
            env.rollout(acts[s][:L], obs[:L], rew[:L], done[:L],
                        partial=partials[s] if stat else None)
        if stat:
            mark[s].record(main_s)
            pending.append((k, s))
            nstat[0] += 1

    trace = [] if args.trace_host else None

    def stamp(what):
        if trace is not None:
            trace.append((what, time.perf_counter()))

    def region(plan, stat_every, evs=None, release_after=None, release=None):
        """The timed region's work: the launches of `plan`, stats on the first launch of every
        `stat_every` (a stats launch's reduction is issued after the next launch, so it runs
        on the side stream under that launch), then the wait for the last stats (side stream /
        all-reduce).  `evs` = (start, end) timing events: start right before the first kernel,
        end right after the last.  No timing event goes between launches: the command processor
        idles the GPU ~12 us at each one (it completes the kernel and writes back the caches
        before it takes the timestamp; rocprofv3 kernel trace, profiles/r5_region_trace.txt),
        where a launch after a plain kernel or a timing-free event starts at once.
        `release` (gated window) is called once launch `release_after` and the reductions issued
        after it are queued, or at the end when that is the last launch."""
        n = len(plan)
        for k, L in enumerate(plan):
            launch(k, L, stat=not args.no_stats and k % stat_every == 0,
                   ev=evs[0] if (evs is not None and k == 0) else None)
            stamp(f"launch {k}")
            if evs is not None and k == n - 1:
                evs[1].record(main_s)
            flush(before=k)
            stamp(f"stats before {k}")
            if release is not None and k == release_after and k < n - 1:
                release()
        flush(last=bool(pending) and pending[-1][0] == n - 1)
        stamp("last stats")
        if release is not None and release_after >= n - 1:
            release()
        # The last stats' buffer; nothing on the device consumes it, so no stream waits for the
        # side stream here: the caller's device-wide synchronize (every stream, RCCL's included)
        # completes it before the host reads it.
        stamp("region issued")
        return None if args.no_stats else stats.bufs[(stats.k - 1) % 2]

    # 1) pre-warm by device time: clocks, first touch of the 2 GB rollout buffer, and the first
    # use of every kernel, stream and event the timed region uses (a kernel's first launch or a
    # stream's first use in a process costs milliseconds of host time -- e.g. the stats
    # reduction kernel, the stats reducer's stream); 2) exactly --warmup steps; 3) exactly
    # --steps timed steps.
    # The number of pre-warm regions is agreed over the ranks (each region holds a stats
    # all-reduce, so every rank must run the same count): one calibration region, then the
    # max over ranks of the regions still needed.
    pw_launches, pw_ms = 0, 0.0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def prewarm_region():
        e0.record(main_s)
        region([T] * 5, 5)
        e1.record(main_s)
        e1.synchronize()
        return e0.elapsed_time(e1)

    # one full collection now, then freeze what survives: the collection right before the timed
    # region then only walks objects made since, instead of idling the GPU for a full
    # generation-2 pass over every torch object (~40 ms) just before the first timed launch
    if not args.no_gc_freeze:
        gc.collect()
        gc.freeze()
    pw_ms += prewarm_region()      # first use of everything (slow)
    last = prewarm_region()        # calibration: one warm region
    pw_ms += last
    pw_launches += 10
    more = int(pdist.max_over_ranks(min(20000, max(0.0, -(-(args.prewarm_ms - pw_ms) //
                                                        max(last, 1e-3)))), dev))
    for _ in range(more):
        pw_ms += prewarm_region()
        pw_launches += 5
    # the timed region's plan and events are made (and each event recorded once) before the
    # closing synchronize, so nothing but the barrier separates the warm-up launches from the
    # first timed launch
    plan = launch_plan(args.steps, T)
    stat_every = max(1, min(args.stats_every, len(plan)))
    # The launch gate (include/fenv.h fenv_stream_gate): a one-wave kernel at the head of the main
    # stream polls a word of device-mapped host memory; the window's launches, stats reductions
    # and all-reduces are issued behind it, then the host takes t0 and stores the word.  Host
    # issue -- and the random 80-250 us stalls inside post-synchronize HIP calls, which 2 of 7
    # processes showed at the 8/4/2-way shard sizes (profiles/r5_shard_sweep_gcfreeze.txt) --
    # leaves the window; every launch's device execution and the closing synchronize stay in it.
    # Plans longer than GATE_PREFIX launches release the gate after the first GATE_PREFIX (the
    # rest is issued while the device runs those: bounded queue depth).  Host-issued instead:
    # MT19937 mode (its refills can wait on the device for a consumed staging slot, which a held
    # stream never frees) and a gloo process group (gloo's wait() on a CUDA tensor's all-reduce
    # blocks the host until the tensor's producer -- held behind the gate -- has run).
    gated = (args.issue == "gated" and args.reset_mode == "philox"
             and (not pdist.active() or torch.distributed.get_backend() == "nccl"))
    gate, gate_error = None, None
    if gated:
        try:
            gate = _Gate(flib, L_abi, dev, main_s)
        except Exception as ex:  # noqa: BLE001 -- the line then carries the host-issued window
            gate_error = f"gate setup: {type(ex).__name__}: {ex}"
        # every rank runs the same windows (each holds collectives)
        gated = pdist.max_over_ranks(0.0 if gate is not None else 1.0, dev) == 0.0

    def window(use_gate: bool):
        """--warmup steps, a synchronize (+ barrier), then one timed window of `plan`."""
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for e in evs:
            e.record(main_s)
        for L in launch_plan(args.warmup, T):
            launch(-1, L)
        torch.cuda.synchronize()
        if pdist.active():
            torch.distributed.barrier()
        torch.cuda.synchronize()
        freed[0] = freed[1] = None  # the synchronize completed every reduction (no wait packets)
        if trace is not None:
            trace.clear()
        # no cyclic-GC pass inside the window (as timeit does): a generation-2 collection over the
        # torch objects alive here takes far longer than the 20-step window.  The objects made
        # before the pre-warm are frozen, so this collection is short: a full one here idled the
        # GPU ~40 ms right before the first timed launch, and the window then ran ~6 % slower
        # (first launches slower, fixed overhead 60 vs 27 us; profiles/ab/r5_gc_freeze_ab.txt)
        gc.collect()
        gc.disable()
        w = {}
        # With a process group, the ranks start their windows at one agreed instant of the node's
        # monotonic clock (one all-reduce before the window): each rank queues its prefix, then
        # spins until that instant.  Otherwise a rank whose host issued faster would start early
        # and then wait, inside its window, for the later ranks' stats all-reduce -- the skew of
        # the ranks' issue times would add to the max over ranks.
        start_at = (int(pdist.max_over_ranks(time.monotonic_ns() + ALIGN_MARGIN_NS, dev))
                    if pdist.active() else None)

        def aligned():
            """Spin to the agreed start (no-op without a process group); record lateness."""
            if start_at is None:
                return
            now = entry = time.monotonic_ns()
            w["start_late_us"] = max(0, now - start_at) / 1e3
            # bounded: ranks on different hosts would not share the clock (bench runs one node)
            while now < start_at and now - entry < 2 * ALIGN_MARGIN_NS:
                now = time.monotonic_ns()

        if use_gate:
            t_arm = time.perf_counter()
            gate.arm()
            rel = min(len(plan), GATE_PREFIX) - 1
            t0 = None

            def release():
                nonlocal t0
                w["prefix_issue_ms"] = (time.perf_counter() - t_arm) * 1e3
                aligned()
                t0 = time.perf_counter()
                # host clocks of the store, to place it on a rocprofv3 kernel trace's time axis
                # (tools/gate_latency.py: store -> gate wave exit -> first launch start)
                w["release_clock_ns"] = {"boottime": time.clock_gettime_ns(time.CLOCK_BOOTTIME),
                                         "monotonic": time.monotonic_ns()}
                gate.release()
                stamp("gate released")

            tot = region(plan, stat_every, evs, release_after=rel, release=release)
        else:
            aligned()
            t0 = time.perf_counter()
            tot = region(plan, stat_every, evs)
        t_issued = time.perf_counter() - t0
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        gc.enable()
        stamp("synchronized")
        w.update(elapsed=elapsed, host_issue_ms=t_issued * 1e3, tot=tot,
                 kern_ms=evs[0].elapsed_time(evs[1]), t0=t0,
                 trace=None if trace is None else [(k, round((t - t0) * 1e6, 2))
                                                   for k, t in trace])
        if use_gate:
            w["gate"] = gate.status()
            w["gate"]["prefix_launches"] = min(len(plan), GATE_PREFIX)
            # released != 1: the gate timed out, so this window is not a measurement; the line
            # then falls back to the host-issued window (below) and says why
        # the closing barrier stays outside the window: max_over_ranks(elapsed) below already takes
        # the slowest rank, and a barrier inside would add a collective's latency to every rank
        if pdist.active():
            torch.distributed.barrier()
        return w

    # the host-issued window first (rounds 1-5's measurement), then the gated one (the headline)
    w_host = window(False)
    w_gate = window(True) if gated else None
    if not args.no_gc_freeze:
        gc.unfreeze()
    if w_gate is not None and pdist.max_over_ranks(
            0.0 if w_gate["gate"]["released"] == 1 else 1.0, dev) != 0.0:
        gate_error = f"gate did not release on every rank: {w_gate['gate']}"
        w_gate = None
    head = w_gate or w_host
    gate_probe = gate.probe() if w_gate is not None else None  # after both windows
    ceiling = hbm_ceiling(acts[0], obs, rew, done, A, T, D, main_s)  # after the timed region
    # the same byte mix over the first 4 planes only: its 0.17 GB of actions stay in the 256 MB
    # Infinity Cache from one k_mix launch to the next, so this is NOT an HBM ceiling -- it shows
    # what the launch's re-read actions cost it (profiles/r5_footprint_ubench.txt)
    ceiling_small = hbm_ceiling(acts[0], obs, rew, done, A, min(T, 4), D, main_s)
    # per-rank timings of both windows (one all-gather), then the max over ranks
    wins = [w for w in (w_host, w_gate) if w is not None]
    mine = [x for w in wins for x in (w["elapsed"] * 1e3, w["kern_ms"], w["host_issue_ms"],
                                      w.get("start_late_us", 0.0))]
    per = pdist.gather_floats(mine, dev)
    per_rank = []
    for i, w in enumerate(wins):
        cols = [[r[4 * i + j] for r in per] for j in range(4)]
        per_rank.append({"elapsed_ms": cols[0], "kernel_ms": cols[1], "host_issue_ms": cols[2],
                         "start_late_us": cols[3]})
        w["elapsed_max"] = max(cols[0]) * 1e-3
        w["kern_ms_max"] = max(cols[1])
    elapsed, kern_total_ms, tot = head["elapsed_max"], head["kern_ms_max"], head["tot"]
    t_issued = head["host_issue_ms"] * 1e-3

    steps = sum(plan)
    kern_avg_ms = kern_total_ms * T / steps  # per T-step launch (equal to the mean when uniform)
    total_agents = total_formations * N
    value = total_agents * steps / elapsed
    # the same agent-steps over the slowest rank's event-timed kernel time: what the kernels
    # scale to with the region's fixed host / synchronisation cost taken out (never `value`)
    kernel_value = total_agents * steps / (kern_total_ms * 1e-3)
    bytes_launch = rollout_bytes_per_launch(A, N, D, T)
    bytes_timed = sum(rollout_bytes_per_launch(A, N, D, L) for L in plan)
    achieved = bytes_timed / (kern_total_ms * 1e-3) / 1e9
    workload = (f"config3: {total_formations} formations x {N} agents "
                f"({F} per GPU x {world}), fused {T}-step rollouts, {args.reset_mode} resets"
                + ("" if world == 1 else f", {scaling} scaling"))
    traffic, tsrc = load_pmc_traffic(workload if world == 1 else "")
    kname = env.rollout_kernel_name(T)
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "agent-steps/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / steps,
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: U(-1,1) fp32 actions resident in HBM, random-init formations",
            "warmup_launches": pw_launches,
            "warmup_ms": pw_ms,
            "host_issue_ms": t_issued * 1e3,
            "kernel_value": kernel_value,
            "fixed_overhead_ms": elapsed * 1e3 - kern_total_ms,
            "issue": "gated" if head is w_gate else "host",
            **({"gate_error": gate_error} if gate_error else {}),
            **({"gate": {**head["gate"], "release_probe": gate_probe,
                         "prefix_issue_ms": head["prefix_issue_ms"],
                         "release_clock_ns": head["release_clock_ns"]}}
               if head is w_gate else {}),
            "host_issued": window_summary(w_host, total_agents, steps),
            **({"per_rank": {"host": per_rank[0],
                             **({"gated": per_rank[1]} if w_gate is not None else {})}}
               if pdist.active() else {}),
            **({"host_trace_us": head["trace"]} if trace is not None else {}),
            "config": {"workload": workload, "formations": total_formations,
                       "agents_per_formation": N, "obs_dim": D, "rollout_chunk": T,
                       "formations_per_gpu": F, "reset_mode": args.reset_mode,
                       "episode_phase": phase,
                       # steps per timed launch: {count, steps} when uniform, else the list
                       "timed_launches": ({"count": len(plan), "steps": plan[0]}
                                          if plan and len(set(plan)) == 1 else plan),
                       "parallelism": f"formation-shard dp{world} ({scaling}: "
                                       + ("formations split over the ranks"
                                          if scaling == "strong" else
                                          f"{F} formations per rank") + ")"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic, "traffic_source": tsrc,
                         "kernel": f"{kname} (fenv_rollout)",
                         "algorithmic_bytes_per_launch": bytes_launch,
                         "algorithmic_bytes_timed": bytes_timed,
                         "avg_kernel_ms": kern_avg_ms, "kernel_ms_timed": kern_total_ms,
                         "launches": len(plan),
                         "timing": "two HIP events on the launch stream, before the first and "
                                   "after the last timed launch (none between launches: each "
                                   "would idle the GPU ~12 us)"},
        }
        if ceiling is not None:
            ceiling["frac_of_spec"] = ceiling["achieved"] / HBM_PEAK_GBS
            ceiling["kernel_frac_of_ceiling"] = (bytes_launch / (kern_avg_ms * 1e-3) / 1e9
                                                 / ceiling["achieved"])
            ceiling["rank"] = 0
            ceiling["footprint"] = ("matched: the launch's own buffers and reuse distance "
                                    f"({bytes_launch / 1e9:.2f} GB per launch), so it shares every "
                                    "footprint-dependent limit of the launch")
            if ceiling_small is not None:
                ceiling["small_footprint"] = {
                    "achieved": ceiling_small["achieved"], "steps": ceiling_small["steps"],
                    "frac_of_spec": ceiling_small["achieved"] / HBM_PEAK_GBS,
                    "note": "k_mix over the first 4 planes only: its 0.17 GB of re-read actions "
                            "stay in the 256 MB Infinity Cache across launches, so this is the "
                            "mix with its reads served from the cache, not an HBM ceiling"}
            out["roofline"]["same_box_ceiling"] = ceiling
        if not args.no_stats:
            t = tot.cpu().tolist()
            sampled = [L for k, L in enumerate(plan) if k % stat_every == 0][-1]
            out["episode_stats"] = {"mean_reward_sampled_rollout": t[0] / (total_agents * sampled),
                                    "agent_dones_sampled_rollout": t[1],
                                    "every_launches": stat_every}
        return out, env
    return None, env


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--formations", type=int, default=1 << 20,
                    help="formations in total (strong scaling, the N > 1 default), or per GPU "
                         "(weak scaling)")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: shard --formations over the ranks (= --scaling strong)")
    ap.add_argument("--scaling", default="auto", choices=["auto", "weak", "strong"],
                    help="auto: strong for N > 1 (BASELINE config 3: 1M formations sharded over "
                         "the GPUs), weak (= strong) at N = 1")
    ap.add_argument("--no-weak-line", action="store_true",
                    help="N > 1: skip the second (other-scaling) measurement nested in the line")
    ap.add_argument("--agents", type=int, default=5)
    ap.add_argument("--chunk", type=int, default=10)
    ap.add_argument("--reset-mode", default="philox", choices=["philox", "mt19937"])
    ap.add_argument("--episode-phase", default="staggered", choices=["staggered", "aligned"],
                    help="staggered (philox only): formations spread over the episode, so every "
                         "window includes resets; aligned: all start at t=0 like the reference")
    ap.add_argument("--no-goal", action="store_true")
    ap.add_argument("--prewarm-ms", type=float, default=400.0,
                    help="device-time pre-warm (clocks, first-touch of the buffers) before the "
                         "--warmup steps; independent of --warmup, reported as warmup_ms")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--issue", default="gated", choices=["gated", "host"],
                    help="gated (philox): the window's launches are queued behind a launch gate "
                         "released at t0, so host issue is outside it; the host-issued window is "
                         "measured too and nested as host_issued.  host: host-issued only")
    ap.add_argument("--no-gc-freeze", action="store_true",
                    help="A/B switch: no gc.freeze() before the pre-warm")
    ap.add_argument("--no-stats", action="store_true")
    ap.add_argument("--trace-host", action="store_true",
                    help="diagnostic: host timestamps (us after t0) of the timed region's calls")
    ap.add_argument("--stats-every", type=int, default=10,
                    help="reduce + all-reduce the episode stats every this many rollout launches "
                         "(clamped to the timed launch count)")
    ap.add_argument("--no-policy", action="store_true", help="skip the config-2 policy rollout")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the secondary env-only lines (BASELINE configs[1] and [4])")
    args = ap.parse_args()
    if args.steps < 1 or args.warmup < 0 or args.chunk < 1:
        ap.error("need --steps >= 1, --warmup >= 0, --chunk >= 1")

    import torch
    import pkgload
    pkg = pkgload.load()
    from importlib import import_module
    pdist = import_module(pkg.__name__ + ".distributed")

    rank, world, local = pdist.init_from_env()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)

    N = args.agents
    D = 6 if args.no_goal else 8
    if args.scaling == "auto":
        scaling = "strong" if world > 1 else "weak"
    else:
        scaling = args.scaling
    if args.strong:
        scaling = "strong"
    # BASELINE config 3 as written: 1,048,576 formations sharded over the GPUs (strong); the
    # weak line (1,048,576 formations on every GPU) rides along as a nested measurement
    total = args.formations if scaling == "strong" else args.formations * world
    out, env = run_config3(args, pkg, rank, world, dev, total, scaling)
    if rank == 0:
        # the collectives of the line (stats all-reduce, barriers, max over ranks): "none" when no
        # process group is up (the driver's N = 1 run); FENV_DIST_FORCE=1 runs them at world 1
        out["dist"] = {"backend": torch.distributed.get_backend() if pdist.active() else "none",
                       "world": world}
    env.release()
    del env
    if world > 1 and not args.no_weak_line:
        other = "weak" if scaling == "strong" else "strong"
        tot2 = args.formations * world if other == "weak" else args.formations
        o2, env2 = run_config3(args, pkg, rank, world, dev, tot2, other)
        env2.release()
        del env2
        if rank == 0:
            keep = ("value", "kernel_value", "fixed_overhead_ms", "ms_per_step", "scaling",
                    "config", "roofline", "steps", "issue", "gate",
                    "host_issued", "per_rank")
            out[f"{other}_scaling_line"] = {k: o2[k] for k in keep if k in o2}
    if rank == 0:
        if world == 1 and not args.no_policy:
            out["policy_rollout"] = secondary(policy_rollout_bench, pkg.__name__, dev, 65536, 10,
                                              10)
        if world == 1 and not args.no_policy:
            out["ppo_update"] = secondary(ppo_update_bench, pkg.__name__, dev)
        if world == 1 and not args.no_configs:
            # the PCIe-inclusive numpy face: the reference's default size (config 0) and the
            # headline size
            out["numpy_face"] = {
                "config0": secondary(numpy_face_bench, pkg.__name__, dev, 1000, N, 200),
                "config3": secondary(numpy_face_bench, pkg.__name__, dev, args.formations, N, 10)}
            out["mt19937_mode"] = secondary(mt_mode_bench, pkg.__name__, dev, args.formations, N)
            out["random_action_rollout"] = random_action_bench(pkg.__name__, dev,
                                                               args.formations, N)
            out["env_configs"] = {"config1": env_config_bench(pkg.__name__, dev, 4096, 5, 400),
                                  "config4": env_config_bench(pkg.__name__, dev, 16384, 64)}
            # the single-step face at the headline size: SURVEY §8(d)'s B_step per agent-step
            out["single_step"] = env_config_bench(pkg.__name__, dev, args.formations, N, 500,
                                                  T=1)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(N, D, args.cpu_baseline_seconds)
        print(json.dumps(out), flush=True)
    if pdist.active():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
