"""Replay the golden fixtures (tests/golden/*.npz) against any env with the FormationEnv face.

The fixtures were produced by the reference itself (tests/golden/gen_golden.py).  An env under
test must provide ``reset() -> obs``, ``step(actions) -> (obs, rew, done, _)`` and
``get_state() -> (px, py, gx, gy, t)`` (numpy); the checks are bit-exact on every byte.
"""
from __future__ import annotations

import glob
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
GOLDEN = os.path.join(HERE, "golden")
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from oracle import synth_actions  # noqa: E402


def d64(*arrs) -> np.uint64:
    h = hashlib.blake2b(digest_size=8)
    for a in arrs:
        h.update(np.ascontiguousarray(a).tobytes())
    return np.frombuffer(h.digest(), dtype=np.uint64)[0]


def case_names():
    return sorted(os.path.splitext(os.path.basename(p))[0]
                  for p in glob.glob(os.path.join(GOLDEN, "*.npz")))


def load_case(name: str) -> dict:
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    d = {k: z[k] for k in z.files}
    F, N, goal, seed, act_seed, steps, log = (int(v) for v in d["meta"])
    d.update(F=F, N=N, goal_in_obs=bool(goal), seed=seed, act_seed=act_seed, steps=steps,
             log=bool(log), A=F * N, amp=float(d["amp"]))
    return d


def _state_vec(px, py, gx, gy):
    ag = np.stack([px, py], axis=1).reshape(-1)
    gl = np.stack([gx, gy], axis=1).reshape(-1)
    return np.concatenate([ag, gl]).astype(np.float32), ag.astype(np.float32), gl.astype(np.float32)


def replay(case: dict, make_env, max_steps: int | None = None, check_state: bool = True):
    """Run ``make_env(case)`` through the fixture; raise AssertionError at the first mismatch.

    ``make_env`` must return an env whose ctor consumed draw set 1 (like FormationEnv)."""
    env = make_env(case)
    A, F = case["A"], case["F"]
    if check_state:
        px, py, gx, gy, t = env.get_state()
        sv, _, _ = _state_vec(px, py, gx, gy)
        assert np.array_equal(sv.view(np.uint32), case["state_ctor"].view(np.uint32)), "ctor state"
    obs = np.asarray(env.reset())
    assert np.array_equal(obs.view(np.uint32), case["obs_reset"].view(np.uint32)), "reset obs"
    if check_state:
        px, py, gx, gy, t = env.get_state()
        sv, _, _ = _state_vec(px, py, gx, gy)
        assert np.array_equal(sv.view(np.uint32), case["state_reset"].view(np.uint32)), "reset state"
    steps = case["steps"] if max_steps is None else min(case["steps"], max_steps)
    sel = {int(s): j for j, s in enumerate(case["sel_steps"])}
    for k in range(1, steps + 1):
        a = synth_actions(case["act_seed"], k, A, case["amp"])
        obs, rew, done, _ = env.step(a)
        obs = np.asarray(obs)
        rew = np.asarray(rew)
        done = np.asarray(done).astype(np.bool_)
        dig = case["digest"][k - 1]
        if k in sel:
            j = sel[k]
            np.testing.assert_array_equal(obs.view(np.uint32), case["sel_obs"][j].view(np.uint32),
                                          err_msg=f"obs step {k}")
            np.testing.assert_array_equal(rew.view(np.uint32), case["sel_rew"][j].view(np.uint32),
                                          err_msg=f"reward step {k}")
            np.testing.assert_array_equal(done, case["sel_done"][j], err_msg=f"done step {k}")
        assert d64(obs) == dig[0], f"obs digest step {k}"
        assert d64(rew) == dig[1], f"reward digest step {k}"
        assert d64(done) == dig[2], f"done digest step {k}"
        if check_state:
            px, py, gx, gy, t = env.get_state()
            _, ag, gl = _state_vec(px, py, gx, gy)
            assert d64(ag) == dig[3], f"agents digest step {k}"
            assert d64(gl, np.asarray(t, np.int32)) == dig[4], f"goal/t digest step {k}"
    return env
