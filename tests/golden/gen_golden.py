"""Generate the golden parity fixtures by importing the REFERENCE env (build container only).

Run from the repo root in the build container (where /root/reference exists):

    PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg python tests/golden/gen_golden.py

The reference (/root/reference/vectorized_env.py, simulate.py) is imported with small stand-in
modules for its absent third-party imports (stable_baselines3, gymnasium, wandb, hydra,
omegaconf -- none is installed and none is on the env-step path; SURVEY.md §8(c) "stub recipe").
The wandb stand-in records every ``wandb.log`` dict so the reference's own logged metrics
(simulate.py:188-208, 251-254; vectorized_env.py:80-81) become fixtures too.

Output: tests/golden/<case>.npz -- DATA only (seeds, shapes, per-step digests, selected full
arrays, logged scalars).  Nothing from the reference's source travels with the repo.

Per case:
  meta            int64 [F, N, goal_in_obs, seed, act_seed, steps, log]
  amp             float64 action amplitude (actions = oracle.synth_actions(act_seed, step, A, amp);
                  amp < 0 selects its edge-case mode)
  d_nb            float32 desired neighbour distance as the reference holds it
  state_ctor      float32 [A*2 + F*2] agents + goal after the ctor (draw set 1)
  obs_reset       float32 [A, D] from env.reset() (draw set 2)
  state_reset     float32 [A*2 + F*2]
  digest          uint64 [steps, 5] blake2b-64 of (obs, reward, done, agents, goal|t bytes)
  sel_steps       int64 [k] 1-based step numbers with full arrays below
  sel_obs/sel_rew/sel_done/sel_agents/sel_goal/sel_t
  rew_sum         float64 [steps] sum of rewards per step (diagnostic)
  log_comp        float32 [steps, 7] formation-0 logged components (if log)
  log_reward      float32 [steps, F] per-formation mean reward (if log)
"""
from __future__ import annotations

import hashlib
import os
import sys
import types

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from oracle import synth_actions  # noqa: E402

LOGS: list = []


def _install_stubs() -> None:
    def mod(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m

    mod("wandb", log=lambda d: LOGS.append(dict(d)), init=lambda **k: None)
    mod("wandb.integration")
    mod("wandb.integration.sb3", WandbCallback=object)

    class VecEnv:
        def __init__(self, num_envs, observation_space, action_space):
            self.num_envs = num_envs
            self.observation_space = observation_space
            self.action_space = action_space

    mod("stable_baselines3")
    mod("stable_baselines3.common")
    mod("stable_baselines3.common.vec_env", VecEnv=VecEnv)
    mod("stable_baselines3.common.callbacks", CheckpointCallback=object)

    class Box:
        def __init__(self, low, high, shape, dtype):
            self.low, self.high, self.shape, self.dtype = low, high, shape, dtype

    sp = mod("gymnasium.spaces", Box=Box)
    mod("gymnasium", spaces=sp)
    mod("hydra", main=lambda **kw: (lambda f: f))
    mod("omegaconf", DictConfig=object, OmegaConf=object)


def _d64(*arrs) -> np.uint64:
    h = hashlib.blake2b(digest_size=8)
    for a in arrs:
        h.update(np.ascontiguousarray(a).tobytes())
    return np.frombuffer(h.digest(), dtype=np.uint64)[0]


CASES = [
    # name,               F,    N,  goal,  seed,       act_seed, steps, amp, log, full_all
    ("f4_n5_d8",          4,    5,  True,  0,          11,       2100,  1.2, True,  False),
    ("f3_n10_d6",         3,    10, False, 1,          12,       1100,  1.0, False, False),
    ("f2_n64_d8",         2,    64, True,  2,          13,       1100,  1.0, True,  False),
    ("f5_n1_d8",          5,    1,  True,  3,          14,       1010,  1.5, True,  False),
    ("f5_n2_d8",          5,    2,  True,  4,          15,       1010,  1.2, True,  False),
    ("f4_n3_d6",          4,    3,  False, 5,          16,       1010,  1.2, False, False),
    ("f1_n5_d8_walls",    1,    5,  True,  7,          17,       2010,  3.0, True,  False),
    ("f16_n7_d8",         16,   7,  True,  123,        18,       1010,  1.2, False, False),
    ("f13_n5_d8_short",   13,   5,  True,  99,         19,       30,    1.2, False, True),
    ("f40_n12_d8_short",  40,   12, True,  2024,       20,       20,    1.2, False, True),
    ("f3_n100_d8",        3,    100, True, 31,         21,       1010,  1.0, False, False),
    ("f2_n33_d6",         2,    33, False, 32,         22,       1010,  1.0, False, False),
    ("f2_n5_seedmax",     2,    5,  True,  2**32 - 1,  23,       50,    1.0, False, True),
    ("default_cfg_f1000", 1000, 5,  True,  0,          24,       3,     1.0, False, True),
    # amp < 0: oracle.synth_actions' "extreme" mode (signed zeros, subnormal, huge, +-inf)
    ("f6_n5_d8_extreme",  6,    5,  True,  77,         25,       1010,  -1.0, True, False),
    ("f4_n3_d6_extreme",  4,    3,  False, 78,         26,       40,    -1.0, False, True),
]

SEL = [1, 2, 3, 500, 1001, 1002, 1003, 2003, 2004, 2005]


def run_case(name, F, N, goal, seed, act_seed, steps, amp, log, full_all):
    import torch
    from types import SimpleNamespace
    import vectorized_env

    torch.manual_seed(seed)
    cfg = SimpleNamespace(num_formation=F, num_agents_per_formation=N, goal_in_obs=goal,
                          share_reward_ratio=0.25, name="golden")
    env = vectorized_env.FormationEnv(cfg, visualize=False, log=log)
    A = F * N

    def state():
        ag = np.concatenate([s.agents.numpy().reshape(-1) for s in env.formationsim_list])
        gl = np.concatenate([s.goal.numpy().reshape(-1) for s in env.formationsim_list])
        t = np.array([s.steps_since_reset for s in env.formationsim_list], np.int32)
        return ag.astype(np.float32), gl.astype(np.float32), t

    ag, gl, _ = state()
    state_ctor = np.concatenate([ag, gl])
    obs_reset = env.reset().copy()
    ag, gl, _ = state()
    state_reset = np.concatenate([ag, gl])

    digest = np.zeros((steps, 5), np.uint64)
    rew_sum = np.zeros(steps)
    sel = [s for s in range(1, steps + 1)] if full_all else [s for s in SEL if s <= steps]
    sel_obs, sel_rew, sel_done, sel_ag, sel_gl, sel_t = [], [], [], [], [], []
    log_comp = np.zeros((steps, 7), np.float32)
    log_rew = np.zeros((steps, F), np.float32)
    comp_keys = ["close_to_goal_reward", "reward_dist", "reward_right_neighbor",
                 "reward_left_neighbor", "avg_dist_to_goal", "ave_dist_to_neighbor",
                 "std_dist_to_neighbor"]
    for k in range(1, steps + 1):
        a = synth_actions(act_seed, k, A, amp)
        LOGS.clear()
        obs, rew, done, infos = env.step(a)
        assert len(infos) == A
        ag, gl, t = state()
        digest[k - 1] = [_d64(obs), _d64(rew), _d64(done), _d64(ag), _d64(gl, t)]
        rew_sum[k - 1] = float(np.sum(rew.astype(np.float64)))
        if k in sel:
            sel_obs.append(obs.copy()); sel_rew.append(rew.copy()); sel_done.append(done.copy())
            sel_ag.append(ag); sel_gl.append(gl); sel_t.append(t)
        if log:
            comp = [d for d in LOGS if "reward" not in d]
            rw = [d["reward"] for d in LOGS if "reward" in d]
            assert len(rw) == F, (len(rw), F)
            got = {}
            for d in comp:
                got.update(d)
            log_comp[k - 1] = [got[c] for c in comp_keys]
            log_rew[k - 1] = rw
    out = dict(
        meta=np.array([F, N, int(goal), seed, act_seed, steps, int(log)], np.int64),
        amp=np.float64(amp),
        d_nb=np.float32(env.formationsim_list[0].desired_neighbor_dist),
        state_ctor=state_ctor, obs_reset=obs_reset, state_reset=state_reset,
        digest=digest, rew_sum=rew_sum, sel_steps=np.array(sel, np.int64),
        sel_obs=np.array(sel_obs, np.float32), sel_rew=np.array(sel_rew, np.float32),
        sel_done=np.array(sel_done, np.bool_), sel_agents=np.array(sel_ag, np.float32),
        sel_goal=np.array(sel_gl, np.float32), sel_t=np.array(sel_t, np.int32),
    )
    if log:
        out["log_comp"] = log_comp
        out["log_reward"] = log_rew
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **out)
    print(f"{name}: F={F} N={N} steps={steps} dones={int(sum(d.any() for d in sel_done))}",
          flush=True)


def main(argv):
    os.environ.setdefault("MPLBACKEND", "Agg")
    sys.dont_write_bytecode = True
    _install_stubs()
    sys.path.insert(0, REF)
    want = set(argv[1:])
    for c in CASES:
        if want and c[0] not in want:
            continue
        run_case(*c)


if __name__ == "__main__":
    main(sys.argv)
