"""CPU oracle for the formation env hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` may
import this module.  It is the checker, never the thing measured or shipped: the product path
(``marl-distributedformation_amd``) runs the HIP library and fails loudly without it.

Two restatements of the same algorithm (reference ``simulate.py:70-236`` and
``vectorized_env.py:22-82``, global torch CPU MT19937 resets ``simulate.py:120-147``):

* :class:`COracleEnv` -- ctypes wrapper of ``oracle/fenv_oracle.c`` (scalar, bit-exact fp32).
* :class:`NumpyOracleEnv` -- vectorised numpy restatement, bit-exact too (fma emulated exactly).

Both are pinned against ``tests/golden/*.npz`` (fixtures produced by importing the reference
itself in the build container, ``tests/golden/gen_golden.py``).

:func:`synth_actions` is the deterministic synthetic action stream every parity test and the
golden generator share (splitmix64 hash of (seed, step, element) -> U(-amp, amp) in fp32).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

W, H = 400.0, 600.0
MAX_STEPS = 1000

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


# ----------------------------------------------------------------------------- actions
def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


# Edge-case action components of the "extreme" mode (amp < 0): the env does not clip actions
# (vectorized_env.py:69-70, quirk Q10), so the step must be exact for signed zeros, subnormal
# moves off a wall, ±inf / huge pushes that clip exactly onto a wall (then stay "out of bounds"
# while zero actions hold it there, quirk Q5).  NaN is not among them: NaN payload bits are not
# an arithmetic result the reference pins.
EXTREME_ACTIONS = np.array([0.0, -0.0, 1e-45, -1e-45, 1e-39, -1e-39, 1e-30, -1e-30, 3e38, -3e38,
                            np.inf, -np.inf, 40.0, -40.0, 1.0, -1.0], np.float32)


def synth_actions(seed: int, step: int, num_agents: int, amp: float = 1.0) -> np.ndarray:
    """Deterministic U(-amp, amp) fp32 actions [num_agents, 2] for (seed, step).  amp < 0 is the
    "extreme" mode: U(-1.2, 1.2) with about half the components replaced by EXTREME_ACTIONS."""
    with np.errstate(over="ignore"):
        base = (np.uint64(seed) * np.uint64(0x9E3779B97F4A7C15)
                + np.uint64(step) * np.uint64(0xD1B54A32D192ED03))
        idx = np.arange(2 * num_agents, dtype=np.uint64)
        z = _splitmix64(base + idx)
    u = (z >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -24)
    a = (u * np.float32(2.0) - np.float32(1.0)) * np.float32(abs(amp) if amp >= 0 else 1.2)
    a = a.astype(np.float32)
    if amp < 0:
        pick = (z & np.uint64(31)).astype(np.int64)  # low bits: independent of u's high bits
        sel = pick < len(EXTREME_ACTIONS)
        a[sel] = EXTREME_ACTIONS[pick[sel]]
    return a.reshape(num_agents, 2)


def philox_actions(act_seed: int, step: int, first_agent: int, num_agents: int) -> np.ndarray:
    """The actions fenv_rollout_random draws in the kernel (include/fenv.h) for global step
    `step` and global agents [first_agent, first_agent + num_agents): component c is
    (w >> 8) / 2^23 - 1 with w = word 2 (step & 1) + c of Philox4x32-10(counter = (agent,
    step >> 1), key = act_seed).  Not a reference behaviour (the reference takes actions from its
    caller); the build's own synthetic-action generator, restated to check the kernel."""
    from policy_oracle import _philox
    g = np.arange(first_agent, first_agent + num_agents, dtype=np.uint64)
    pair = np.uint64(step >> 1)
    M = np.uint64(0xFFFFFFFF)
    ctr = np.stack([g & M, g >> np.uint64(32), np.full_like(g, pair & M),
                    np.full_like(g, pair >> np.uint64(32))], axis=1)
    w = _philox(ctr, (act_seed & 0xFFFFFFFF, (act_seed >> 32) & 0xFFFFFFFF))
    w = w[:, 2:4] if step & 1 else w[:, 0:2]
    v = (w >> np.uint64(8)).astype(np.int64) - (1 << 23)
    return (v.astype(np.float32) * np.float32(2.0 ** -23)).astype(np.float32)


PHILOX_RESET_KEY1 = 0x5EEDF00D  # fenv_api.cpp fenv_create: c.key1


def philox_reset_draws(seed: int, formations: np.ndarray, num_agents: int,
                       episodes: np.ndarray):
    """The reset draw of ``reset_mode="philox"`` (csrc/env_device.h draw_reset, Philox branch)
    for global formations ``formations`` [k] entering episode ``episodes`` [k] (the formation's
    episode counter after the reset: 1 for the ctor's reset, +1 per reset since).  Same
    distributions as the reference's reset (simulate.py:133-143: agents U(0,400) x U(0,100), goal
    U(60,340) x U(60,540), torch.rand's 24-bit floats), drawn from Philox4x32-10 with key
    (seed, 0x5EEDF00D) instead of the global MT19937 stream:
      agent g = f * N + i: counter (g lo, g hi, episode, 'AGNT') -> words x, y -> px, py;
      formation f:         counter (f lo, f hi, episode, 'GOAL') -> words x, y -> gx, gy.
    Not a reference behaviour (the reference only has the MT19937 stream, which
    ``reset_mode="mt19937"`` replays); the build's throughput-mode RNG, restated to check the
    kernel.  Returns px, py [k * N] and gx, gy [k] (float32, exactly the kernel's roundings:
    one fp32 multiply, and for the goal one multiply then one add)."""
    from policy_oracle import _philox
    M = np.uint64(0xFFFFFFFF)
    f = np.asarray(formations, np.uint64)
    ep = np.asarray(episodes, np.uint64) & M
    N = int(num_agents)
    key = (int(seed) & 0xFFFFFFFF, PHILOX_RESET_KEY1)
    g = (f[:, None] * np.uint64(N) + np.arange(N, dtype=np.uint64)).reshape(-1)
    epa = np.repeat(ep, N)
    ra = _philox(np.stack([g & M, g >> np.uint64(32), epa, np.full_like(g, 0x41474E54)], 1), key)
    rg = _philox(np.stack([f & M, f >> np.uint64(32), ep, np.full_like(f, 0x474F414C)], 1), key)

    def u24(w):
        return (w & np.uint64(0xFFFFFF)).astype(np.float32) * np.float32(2.0 ** -24)

    px = (u24(ra[:, 0]) * np.float32(400.0)).astype(np.float32)
    py = (u24(ra[:, 1]) * np.float32(100.0)).astype(np.float32)
    gx = (u24(rg[:, 0]) * np.float32(280.0) + np.float32(60.0)).astype(np.float32)
    gy = (u24(rg[:, 1]) * np.float32(480.0) + np.float32(60.0)).astype(np.float32)
    return px, py, gx, gy


# ----------------------------------------------------------------------------- MT19937
def mt_raw(seed: int, n: int, skip: int = 0) -> np.ndarray:
    """Raw 32-bit MT19937 outputs after init_genrand(seed) (== torch.manual_seed stream)."""
    bg = np.random.MT19937()
    bg._legacy_seeding(int(seed) & 0xFFFFFFFF)
    if skip:
        bg.random_raw(skip)
    return bg.random_raw(n).astype(np.uint32)


def torch_rand_from_raw(raw: np.ndarray) -> np.ndarray:
    return (raw & np.uint32(0xFFFFFF)).astype(np.float32) * np.float32(2.0 ** -24)


def mt_reset_draws(seed: int, sets, total: int, formations: np.ndarray, num_agents: int):
    """The reference's reset draws for selected formations, straight from the global MT19937
    stream (numpy's MT19937 with init_genrand seeding == torch.manual_seed, vectorized_env.py:
    52-55): draw set s of a ``total``-formation env is the stream's words
    [s * total * (2N + 2), (s + 1) * total * (2N + 2)), formation f's part of it the 2N + 2 words
    from f * (2N + 2) on -- N (x, y) pairs, then the goal pair (simulate.py:133-143, torch.rand =
    (u32 & 0xFFFFFF) * 2^-24; x * 400, y * 100, goal (x * 280 + 60, y * 480 + 60)).  Set 0 is the
    constructor's reset, 1 the first reset(), then one set per timeout.  Independent of the
    library's block-twisted generator and its draw-ahead thread (fenv_api.cpp), which it checks.
    Returns {s: (px [k * N], py [k * N], gx [k], gy [k])} for every s in ``sets``."""
    N = int(num_agents)
    per = 2 * N + 2
    f = np.asarray(formations, np.int64)
    bg = np.random.MT19937()
    bg._legacy_seeding(int(seed) & 0xFFFFFFFF)
    out = {}
    want = sorted(set(int(s) for s in sets))
    cols = (f[:, None] * per + np.arange(per)).reshape(-1)
    for s in range(want[-1] + 1):
        raw = bg.random_raw(total * per)  # one whole set (the stream continues across calls)
        if s not in want:
            continue
        u = torch_rand_from_raw(raw[cols].astype(np.uint32)).reshape(len(f), per)
        px = (u[:, 0:2 * N:2] * np.float32(400.0)).astype(np.float32).reshape(-1)
        py = (u[:, 1:2 * N:2] * np.float32(100.0)).astype(np.float32).reshape(-1)
        gx = (u[:, 2 * N] * np.float32(280.0) + np.float32(60.0)).astype(np.float32)
        gy = (u[:, 2 * N + 1] * np.float32(480.0) + np.float32(60.0)).astype(np.float32)
        out[s] = (px, py, gx, gy)
        del raw
    return out


# ----------------------------------------------------------------------------- exact fmaf
def fmaf(a: np.ndarray, b: np.ndarray, c: np.ndarray) -> np.ndarray:
    """Correctly rounded fp32 fma(a, b, c) for fp32 arrays (one rounding, like v_fma_f32)."""
    a64, b64, c64 = (np.asarray(v, np.float32).astype(np.float64) for v in (a, b, c))
    p = a64 * b64                      # exact: 24x24-bit product fits in 53 bits
    s = p + c64
    bb = s - p                          # TwoSum: p + c64 == s + e exactly
    e = (p - (s - bb)) + (c64 - bb)
    r = s.astype(np.float32)
    r64 = r.astype(np.float64)
    inexact = (r64 != s) & (e != 0)
    if np.any(inexact):
        toward = np.where(s > r64, np.float32(np.inf), np.float32(-np.inf))
        n = np.nextafter(r, toward.astype(np.float32))
        mid = (r64 + n.astype(np.float64)) * 0.5
        tie = inexact & (s == mid)
        # at an exact double tie the true value lies on e's side
        go_n = tie & ((e > 0) == (n.astype(np.float64) > r64))
        r = np.where(go_n, n, r)
    return r.astype(np.float32)


def norm2(x: np.ndarray, y: np.ndarray) -> np.ndarray:
    """torch CPU linalg.norm(dim=1) of 2-vectors == sqrtf(fmaf(y, y, x*x))."""
    x = np.asarray(x, np.float32)
    y = np.asarray(y, np.float32)
    return np.sqrt(fmaf(y, y, x * x)).astype(np.float32)


def desired_neighbor_dist(n: int) -> np.float32:
    """simulate.py:26, rounded to fp32 when it meets the fp32 tensor (simulate.py:202-203)."""
    return np.float32(2 * 60 * np.sin(np.pi / n))


# ----------------------------------------------------------------------------- numpy env
class NumpyOracleEnv:
    """Vectorised restatement of FormationEnv (vectorized_env.py:16-82) over [F, N] arrays."""

    def __init__(self, num_formation: int, num_agents: int, goal_in_obs: bool = True,
                 seed: int = 0, share: float = 0.25, max_steps: int = MAX_STEPS):
        self.F, self.N = int(num_formation), int(num_agents)
        self.goal_in_obs = bool(goal_in_obs)
        self.D = 8 if goal_in_obs else 6
        self.max_steps = int(max_steps)
        self.c_self = np.float32(1.0 - 2 * share)
        self.c_nb = np.float32(share)
        self.d_nb = desired_neighbor_dist(self.N)
        self._bg = np.random.MT19937()
        self._bg._legacy_seeding(int(seed) & 0xFFFFFFFF)
        self.p = np.zeros((self.F, self.N, 2), np.float32)
        self.g = np.zeros((self.F, 2), np.float32)
        self.t = np.zeros(self.F, np.int32)
        self.comp = np.zeros((self.F, 4))
        self._reset_formations(np.arange(self.F))      # ctor draw set (simulate.py:61)
        self.comp = self._components(self.p)

    # simulate.py:120-147, drawn in formation order
    def _reset_formations(self, idx: np.ndarray) -> None:
        k = len(idx)
        if k == 0:
            return
        per = 2 * self.N + 2
        u = torch_rand_from_raw(self._bg.random_raw(k * per).astype(np.uint32)).reshape(k, per)
        ua = u[:, :2 * self.N].reshape(k, self.N, 2)
        self.p[idx, :, 0] = ua[:, :, 0] * np.float32(400)
        self.p[idx, :, 1] = ua[:, :, 1] * np.float32(100)
        self.g[idx, 0] = u[:, -2] * np.float32(280) + np.float32(60)
        self.g[idx, 1] = u[:, -1] * np.float32(480) + np.float32(60)
        self.t[idx] = 0

    def observe(self) -> np.ndarray:
        n = self.p / np.array([W, H], np.float32)
        prev = np.roll(n, 1, axis=1)
        nxt = np.roll(n, -1, axis=1)
        parts = [n, prev - n, nxt - n]
        if self.goal_in_obs:
            parts.append((self.g[:, None, :] - self.p) / np.array([W, H], np.float32))
        return np.concatenate(parts, axis=2).reshape(self.F * self.N, self.D).astype(np.float32)

    def reset(self) -> np.ndarray:
        self._reset_formations(np.arange(self.F))
        self.comp = self._components(self.p)
        return self.observe()

    def _components(self, p: np.ndarray) -> np.ndarray:
        """Per-formation means (float64, agent order) of close_to_goal_reward, reward_dist,
        reward_right_neighbor, reward_left_neighbor (simulate.py:183-208) for positions p."""
        dg = norm2(p[..., 0] - self.g[:, None, 0], p[..., 1] - self.g[:, None, 1])
        pr, pl = np.roll(p, -1, axis=1), np.roll(p, 1, axis=1)
        dr = norm2(p[..., 0] - pr[..., 0], p[..., 1] - pr[..., 1]) - self.d_nb
        dl = norm2(p[..., 0] - pl[..., 0], p[..., 1] - pl[..., 1]) - self.d_nb
        parts = [np.where(dg < np.float32(100), np.float32(10), np.float32(0)),
                 np.float32(-0.1) * dg,
                 np.float32(-0.01) * np.where(dr < 0, dr * dr, dr),
                 np.float32(-0.01) * np.where(dl < 0, dl * dl, dl)]
        out = np.zeros((self.F, 4))
        for k, v in enumerate(parts):
            acc = np.zeros(self.F)
            for i in range(self.N):  # agent order, as the C oracle and the kernel
                acc += v[:, i].astype(np.float64)
            out[:, k] = acc / self.N
        return out

    def step(self, actions: np.ndarray):
        a = np.asarray(actions, np.float32).reshape(self.F, self.N, 2)
        p = self.p + np.float32(10) * a
        oob = ((p[..., 0] <= 0) | (p[..., 1] <= 0) | (p[..., 0] >= np.float32(W))
               | (p[..., 1] >= np.float32(H)))
        p[..., 0] = np.where(p[..., 0] < 0, np.float32(0),
                             np.where(p[..., 0] > np.float32(W), np.float32(W), p[..., 0]))
        p[..., 1] = np.where(p[..., 1] < 0, np.float32(0),
                             np.where(p[..., 1] > np.float32(H), np.float32(H), p[..., 1]))
        self.p = p.astype(np.float32)
        self.comp = self._components(self.p)
        dg = norm2(p[..., 0] - self.g[:, None, 0], p[..., 1] - self.g[:, None, 1])
        ctg = np.where(dg < np.float32(100), np.float32(10), np.float32(0))
        rd = np.float32(-0.1) * dg
        pr = np.roll(p, -1, axis=1)
        pl = np.roll(p, 1, axis=1)
        dr = norm2(p[..., 0] - pr[..., 0], p[..., 1] - pr[..., 1]) - self.d_nb
        dl = norm2(p[..., 0] - pl[..., 0], p[..., 1] - pl[..., 1]) - self.d_nb
        rr = np.float32(-0.01) * np.where(dr < 0, dr * dr, dr)
        rl = np.float32(-0.01) * np.where(dl < 0, dl * dl, dl)
        ind = ((rd + ctg) + rr) + rl
        ind = ind + (np.where(oob, np.float32(-100), np.float32(-0.0)) + np.float32(-0.0))
        rew = (self.c_self * ind
               + self.c_nb * (np.roll(ind, 1, axis=1) + np.roll(ind, -1, axis=1)))
        done_f = self.t > self.max_steps
        self.t = self.t + 1
        self._reset_formations(np.nonzero(done_f)[0])
        done = np.repeat(done_f, self.N)
        return (self.observe(), rew.astype(np.float32).reshape(-1), done,
                None)

    def metrics(self, rew: np.ndarray | None = None) -> np.ndarray:
        """Per-formation [avg_dist_to_goal, mean right-neighbour dist, its unbiased std,
        mean reward] (simulate.py:238-254, vectorized_env.py:80-81), float64."""
        p = self.p.astype(np.float32)
        dg = norm2(p[..., 0] - self.g[:, None, 0], p[..., 1] - self.g[:, None, 1]).astype(np.float64)
        pr = np.roll(p, -1, axis=1)
        dr = norm2(p[..., 0] - pr[..., 0], p[..., 1] - pr[..., 1]).astype(np.float64)
        out = np.zeros((self.F, 8))
        out[:, 4:] = self.comp
        out[:, 0] = dg.mean(1)
        out[:, 1] = dr.mean(1)
        out[:, 2] = dr.std(1, ddof=1) if self.N > 1 else np.nan
        out[:, 3] = 0.0 if rew is None else np.asarray(rew, np.float64).reshape(self.F, self.N).mean(1)
        return out

    def get_state(self):
        return (self.p[..., 0].reshape(-1).copy(), self.p[..., 1].reshape(-1).copy(),
                self.g[:, 0].copy(), self.g[:, 1].copy(), self.t.copy())


# ----------------------------------------------------------------------------- C oracle
_lib = None


def load_lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run `make -C oracle`")
        lib = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        lib.orc_env_create.restype = P
        lib.orc_env_create.argtypes = [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                       ctypes.c_double, ctypes.c_int32, ctypes.c_uint32]
        lib.orc_env_destroy.argtypes = [P]
        lib.orc_env_reset.argtypes = [P, P]
        lib.orc_env_observe.argtypes = [P, P]
        lib.orc_env_step.argtypes = [P, P, P, P, P]
        lib.orc_env_metrics.argtypes = [P, P, P]
        lib.orc_env_get_state.argtypes = [P, P, P, P, P, P]
        lib.orc_env_set_state.argtypes = [P, P, P, P, P, P]
        lib.orc_env_d_nb.argtypes = [P]
        lib.orc_env_d_nb.restype = ctypes.c_float
        lib.orc_mt_raw.argtypes = [ctypes.c_uint32, ctypes.c_uint64, P, ctypes.c_int64]
        _lib = lib
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


class COracleEnv:
    """ctypes wrapper of fenv_oracle.c with the FormationEnv surface (numpy in/out)."""

    def __init__(self, num_formation: int, num_agents: int, goal_in_obs: bool = True,
                 seed: int = 0, share: float = 0.25, max_steps: int = MAX_STEPS):
        self.lib = load_lib()
        self.F, self.N = int(num_formation), int(num_agents)
        self.D = 8 if goal_in_obs else 6
        self.A = self.F * self.N
        self.h = self.lib.orc_env_create(self.F, self.N, int(bool(goal_in_obs)), float(share),
                                         int(max_steps), int(seed) & 0xFFFFFFFF)
        self.obs = np.zeros((self.A, self.D), np.float32)
        self.rew = np.zeros(self.A, np.float32)
        self.done = np.zeros(self.A, np.bool_)

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            self.lib.orc_env_destroy(h)
            self.h = None

    def reset(self) -> np.ndarray:
        self.lib.orc_env_reset(self.h, _ptr(self.obs))
        return self.obs.copy()

    def observe(self) -> np.ndarray:
        self.lib.orc_env_observe(self.h, _ptr(self.obs))
        return self.obs.copy()

    def step(self, actions: np.ndarray):
        a = np.ascontiguousarray(actions, np.float32).reshape(self.A, 2)
        self.lib.orc_env_step(self.h, _ptr(a), _ptr(self.obs), _ptr(self.rew), _ptr(self.done))
        return self.obs.copy(), self.rew.copy(), self.done.copy(), None

    def step_inplace(self, actions: np.ndarray) -> None:
        """Same as step() without the copies (for timing the CPU baseline)."""
        self.lib.orc_env_step(self.h, _ptr(actions), _ptr(self.obs), _ptr(self.rew),
                              _ptr(self.done))

    def metrics(self, rew: np.ndarray | None = None) -> np.ndarray:
        """[F, 8]: compute_metrics (3), mean reward, reward components of the last scored state
        (see fenv_oracle.c orc_env_metrics)."""
        out = np.zeros((self.F, 8), np.float64)
        r = None if rew is None else np.ascontiguousarray(rew, np.float32)
        self.lib.orc_env_metrics(self.h, None if r is None else _ptr(r), _ptr(out))
        return out

    def get_state(self):
        px = np.zeros(self.A, np.float32)
        py = np.zeros(self.A, np.float32)
        gx = np.zeros(self.F, np.float32)
        gy = np.zeros(self.F, np.float32)
        t = np.zeros(self.F, np.int32)
        self.lib.orc_env_get_state(self.h, _ptr(px), _ptr(py), _ptr(gx), _ptr(gy), _ptr(t))
        return px, py, gx, gy, t

    def set_state(self, px, py, gx, gy, t) -> None:
        arrs = [np.ascontiguousarray(v, np.float32) for v in (px, py, gx, gy)]
        tt = np.ascontiguousarray(t, np.int32)
        self.lib.orc_env_set_state(self.h, *[_ptr(v) for v in arrs], _ptr(tt))

    @property
    def d_nb(self) -> float:
        return float(self.lib.orc_env_d_nb(self.h))


def c_mt_raw(seed: int, n: int, skip: int = 0) -> np.ndarray:
    out = np.zeros(n, np.uint32)
    load_lib().orc_mt_raw(int(seed) & 0xFFFFFFFF, int(skip), _ptr(out), int(n))
    return out
