"""FormationEnv: drop-in for the reference's SB3 VecEnv (vectorized_env.py:16-109) on MI355X.

Same constructor, attributes, methods and error behaviour as the reference class, with all F*N
agents stepped by the gfx950 kernels of libfenv.so in one launch per call:

=========================  ===================================================================
reference                  here
=========================  ===================================================================
``FormationEnv(cfg, visualize=False, log=True)``  (:22-50)   same; extra keyword-only knobs
``num_envs``, ``observation_space``, ``action_space``, ``obs_dim``,
``num_agents_per_formation``, ``formationsim_list``           same (views, see simulate.py)
``reset() -> np.float32[A, D]``  (:52-55)                     same (host copy of the device obs)
``step(actions) -> (obs, rew, done, infos)``  (:68-82)       same; arrays alias env buffers
``close/env_is_wrapped/set_attr/env_method/seed/step_async/step_wait`` raise NotImplementedError
``get_attr`` raises AttributeError                             same
=========================  ===================================================================

Device faces (no PCIe per step): :meth:`step_tensor`, :meth:`rollout`, :meth:`observe_tensor`,
:meth:`metrics`, :meth:`get_state` / :meth:`set_state`.

Parity: with ``reset_mode="mt19937"`` (default) and ``seed=s`` the env reproduces, bit for bit,
the reference constructed right after ``torch.manual_seed(s)`` (tests/test_gpu_parity.py).
"""
from __future__ import annotations

import ctypes
from collections.abc import Sequence

import numpy as np
import torch

from . import _lib
from .config import as_config
from .simulate import FormationView, FormationViewList


class Box:
    """Minimal stand-in for ``gymnasium.spaces.Box`` (vectorized_env.py:34-35)."""

    def __init__(self, low, high, shape, dtype):
        self.low = np.full(shape, low, dtype=dtype)
        self.high = np.full(shape, high, dtype=dtype)
        self.shape = tuple(shape)
        self.dtype = np.dtype(dtype)

    def __repr__(self):
        return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"


def _make_box(low, high, shape, dtype):
    try:  # the real gymnasium space when it is installed (SB3 checks isinstance)
        from gymnasium import spaces
        return spaces.Box(low=low, high=high, shape=shape, dtype=dtype)
    except Exception:
        return Box(low, high, shape, dtype)


class _Infos(Sequence):
    """``infos`` list of length A: one empty dict per agent, created on first access."""

    def __init__(self, n: int):
        self._n = int(n)
        self._d: dict[int, dict] = {}

    def __len__(self):
        return self._n

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(self._n))]
        i = int(i)
        if i < 0:
            i += self._n
        if not 0 <= i < self._n:
            raise IndexError(i)
        d = self._d.get(i)
        if d is None:
            d = self._d[i] = {}
        return d


def _vecenv_base():
    """stable-baselines3's ``VecEnv`` when it is importable (the reference's base class,
    vectorized_env.py:16), so ``PPO('MlpPolicy', env)`` accepts the env as a vectorised env;
    ``object`` otherwise (SB3 is not installed in this image)."""
    try:
        from stable_baselines3.common.vec_env import VecEnv
        return VecEnv
    except Exception:
        return object


_BASE = _vecenv_base()


class FormationEnv(_BASE):
    """Batched formation env on one HIP device (one shard of a multi-GPU batch)."""

    MAX_SPEED = 10  # vectorized_env.py:69

    def __init__(self, cfg, visualize: bool = False, log: bool = True, *, device=None,
                 seed: int | None = None, reset_mode: str | None = None,
                 max_steps: int | None = None, honor_share_reward_ratio: bool = False,
                 first_formation: int = 0, total_formations: int | None = None):
        cfg = as_config(cfg)
        self.cfg = cfg
        self.num_agents_per_formation = int(cfg.num_agents_per_formation)
        self.num_formation = int(cfg.num_formation)
        self.goal_in_obs = bool(cfg.goal_in_obs)
        self.obs_dim = 8 if self.goal_in_obs else 6          # vectorized_env.py:28-31
        num_envs = self.num_agents_per_formation * self.num_formation          # :32
        action_space = _make_box(-1, 1, (2,), np.float32)                    # :34
        observation_space = _make_box(-1, 1, (self.obs_dim,), np.float32)   # :35
        if _BASE is not object:  # SB3 VecEnv base: the reference's super().__init__, :36
            super().__init__(num_envs=num_envs, observation_space=observation_space,
                             action_space=action_space)
        self.num_envs = num_envs
        self.action_space = action_space
        self.observation_space = observation_space
        self.device = _lib.require_device(device if device is not None else cfg.get("device"))
        # Q1: the reference never forwards cfg.share_reward_ratio (vectorized_env.py:43)
        self.share_reward_ratio = (float(cfg.share_reward_ratio) if honor_share_reward_ratio
                                   else 0.25)
        self.max_steps = int(max_steps if max_steps is not None else cfg.get("max_steps", 1000))
        if seed is None:
            seed = cfg.get("seed", None)
        if seed is None:  # the torch global stream the reference draws from (simulate.py:133)
            seed = torch.initial_seed()
        self.rng_seed = int(seed) & 0xFFFFFFFF
        mode = reset_mode or cfg.get("reset_mode", "mt19937")
        if mode not in _lib.RESET_MODES:
            raise ValueError(f"reset_mode must be one of {sorted(_lib.RESET_MODES)}")
        self.reset_mode = mode
        self.first_formation = int(first_formation)
        self.total_formations = int(total_formations or self.num_formation)
        self.visualize = bool(visualize)
        self.log = bool(log)
        self.desired_neighbor_dist = float(
            _lib.lib().fenv_desired_neighbor_dist(self.num_agents_per_formation))

        L = _lib.lib()
        _lib.flush_deferred()
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(L.fenv_create(ctypes.byref(h), self.device.index, self.num_formation,
                                     self.num_agents_per_formation, int(self.goal_in_obs),
                                     self.share_reward_ratio, self.max_steps, self.rng_seed,
                                     _lib.RESET_MODES[mode], self.first_formation,
                                     self.total_formations), "fenv_create")
        self._h = h
        self._npartial = int(L.fenv_partial_count(h))
        A, D, F = self.num_envs, self.obs_dim, self.num_formation
        dev = self.device
        # the device faces' default outputs (reset_tensor / observe_tensor / step_tensor); the
        # numpy faces write their own host arrays instead (_ensure_host), so these hold the last
        # device-face results, not necessarily the last step's
        self.obs_dev = torch.zeros((A, D), dtype=torch.float32, device=dev)
        self.rew_dev = torch.zeros(A, dtype=torch.float32, device=dev)
        self.done_dev = torch.zeros(A, dtype=torch.bool, device=dev)
        self._host = None  # zero-copy host arrays of the numpy faces, created on first use
        self.infos = _Infos(A)                                # vectorized_env.py:49
        self.formationsim_list = FormationViewList(self, F)  # vectorized_env.py:38
        self._fig = None
        if self.visualize:
            from .viz import FormationFigure
            self._fig = FormationFigure(self.num_agents_per_formation)
            self._refresh_fig()

    # ------------------------------------------------------------------ plumbing
    def _stream(self):
        return _lib.current_stream(self.device)

    def release(self) -> None:
        """Free this env's device state and staging buffers now, and drop its host arrays (their
        block goes back to the pool once no returned array views it).

        Idempotent.  Afterwards every device call raises.  The reference has no such path: its
        ``close()`` raises NotImplementedError (vectorized_env.py:87-88), which is kept, so this
        is the deterministic teardown (also ``with FormationEnv(cfg) as env: ...``).  Without it
        the env is freed when its last reference goes (views hold only weak references), or --
        for a handle dropped while a HIP graph is being captured -- at the next create/release
        (``_lib.destroy_handle``)."""
        h = getattr(self, "_h", None)
        self._h = None
        if h is not None and h.value:
            if torch.cuda.is_current_stream_capturing():
                # inside a HIP graph capture a synchronize would invalidate it: park the handle
                # (destroyed at the next create / release outside a capture); the torch buffers
                # below are freed by the caching allocator, which defers reuse past the capture
                _lib.destroy_handle(h)
            else:
                # finish the work this env queued on the caller's stream before its buffers go
                torch.cuda.current_stream(self.device).synchronize()
                _lib.destroy_handle(h)
        self._host = None
        for k in ("obs_dev", "rew_dev", "done_dev"):
            if hasattr(self, k):
                setattr(self, k, None)

    @property
    def released(self) -> bool:
        return getattr(self, "_h", None) is None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.release()
        return False

    def __del__(self):
        h = getattr(self, "_h", None)
        self._h = None
        if h is not None and h.value:
            try:
                _lib.destroy_handle(h)
            except Exception:
                pass

    def _ensure_host(self) -> _lib.HostBlock:
        """The numpy faces' arrays (vectorized_env.py:46-48 obs_buf / reward_buf / done_buf, plus
        the actions) in device-mapped host memory: the kernels read the actions and write the
        outputs there directly, so a numpy step is one launch and a synchronize."""
        if self._host is None:
            A, D = self.num_envs, self.obs_dim
            self._host = _lib.HostBlock(self.device, [("act", np.float32, (A, 2)),
                                                      ("obs", np.float32, (A, D)),
                                                      ("rew", np.float32, (A,)),
                                                      ("done", np.bool_, (A,))])
        return self._host

    def _make_view(self, i: int) -> FormationView:
        v = FormationView(self, i)
        if i == 0 and self._fig is not None:
            v.visualize = True
            v.fig = self._fig.fig
            v.ax = self._fig.ax
        return v

    def _formation_state(self, i: int):
        """Formation i's state on the host, copying only its N agents (fenv_get_state_range)."""
        px, py, gx, gy, t = self.get_state_range(i, 1)
        px, py, gx, gy, t = (v.cpu().numpy() for v in (px, py, gx, gy, t))
        return px, py, float(gx[0]), float(gy[0]), int(t[0])

    def _refresh_fig(self):
        if self._fig is None:
            return
        px, py, gx, gy, _ = self._formation_state(0)
        self._fig.update(px, py, gx, gy)

    def check(self) -> None:
        """Raise FenvError if a launch of this env applied a staged MT19937 reset set that failed
        its tag check (``fenv_status``; a host read, no GPU call -- call it after a synchronize
        to cover the launches issued so far).  The numpy faces call it after their copies."""
        _lib.check(_lib.lib().fenv_status(self._h), "fenv_status")

    def info(self) -> dict:
        out = (ctypes.c_int64 * 8)()
        _lib.check(_lib.lib().fenv_info(self._h, out), "fenv_info")
        keys = ["num_formation", "num_agents", "obs_dim", "num_agents_total",
                "steps_since_reset", "reset_mode", "first_formation", "total_formations"]
        return dict(zip(keys, list(out)))

    # ------------------------------------------------------------------ reference API
    def reset(self) -> np.ndarray:
        """vectorized_env.py:52-55: reset every formation and return obs [A, D] (numpy, written in
        place by the kernel; aliases this env's host array like the reference's obs_buf)."""
        host = self._ensure_host()
        _lib.check(_lib.lib().fenv_reset(self._h, host.dev("obs"), self._stream()), "fenv_reset")
        return self._host_result(host).obs

    def compute_observations(self) -> np.ndarray:
        """vectorized_env.py:57-66 (numpy view of the current observations)."""
        host = self._ensure_host()
        _lib.check(_lib.lib().fenv_observe(self._h, host.dev("obs"), self._stream()),
                   "fenv_observe")
        return self._host_result(host).obs

    def step(self, actions):
        """vectorized_env.py:68-82.  ``actions`` [A, 2] in the action space (numpy or tensor).

        Returns ``(obs, rewards, dones, infos)`` as numpy arrays that alias this env's host
        buffers (overwritten by the next call, like the reference's ``obs_buf.numpy()``)."""
        host = self._ensure_host()
        if isinstance(actions, torch.Tensor) and actions.is_cuda:
            act = self._check_act(actions, ())
            act_p = _lib.ptr(act)
        else:
            a = np.asarray(actions, dtype=np.float32)
            if a.shape != (self.num_envs, 2):
                # simulate.py:79 asserts input_velocity.shape == agents.shape per formation
                raise AssertionError(f"actions shape {a.shape} != {(self.num_envs, 2)}")
            np.copyto(host.act, a)
            act_p = host.dev("act")
        _lib.check(_lib.lib().fenv_step(self._h, act_p, host.dev("obs"), host.dev("rew"),
                                        host.dev("done"), self._stream()), "fenv_step")
        self._host_result(host)
        return host.obs, host.rew, host.done, self.infos

    def close(self):
        raise NotImplementedError

    def env_is_wrapped(self, wrapper_class):
        raise NotImplementedError

    def get_attr(self, attr_name, indices=None):
        raise AttributeError

    def set_attr(self, attr_name, value, indices=None):
        raise NotImplementedError

    def env_method(self, method_name, *method_args, indices=None, **method_kwargs):
        raise NotImplementedError

    def seed(self, seed=None):
        raise NotImplementedError

    def step_wait(self):
        raise NotImplementedError

    def step_async(self, actions):
        raise NotImplementedError

    # ------------------------------------------------------------------ device faces
    def _host_result(self, host: _lib.HostBlock) -> _lib.HostBlock:
        """Wait for the launch that writes the host arrays, then the faces' common tail."""
        torch.cuda.current_stream(self.device).synchronize()
        self.check()
        if self._fig is not None:
            self._refresh_fig()
        return host

    def reset_tensor(self) -> torch.Tensor:
        """Reset every formation; returns the device obs buffer [A, D]."""
        _lib.check(_lib.lib().fenv_reset(self._h, _lib.ptr(self.obs_dev), self._stream()),
                   "fenv_reset")
        return self.obs_dev

    def observe_tensor(self) -> torch.Tensor:
        _lib.check(_lib.lib().fenv_observe(self._h, _lib.ptr(self.obs_dev), self._stream()),
                   "fenv_observe")
        return self.obs_dev

    def _on_device(self, t) -> bool:
        return isinstance(t, torch.Tensor) and t.is_cuda and t.get_device() == self.device.index

    def _check_out(self, name: str, t, shape: tuple, dtype) -> None:
        """Caller-supplied output buffers go to the kernels as raw pointers: check them first."""
        if t is None:
            return
        if not self._on_device(t):
            raise ValueError(f"{name} must be a tensor on {self.device}")
        if t.shape != shape or t.dtype != dtype or not t.is_contiguous():
            raise ValueError(f"{name} must be a contiguous {dtype} tensor of shape {tuple(shape)}, "
                             f"got {t.dtype} {tuple(t.shape)}")

    def _check_partial(self, partial) -> None:
        if partial is None:
            return
        n = self._npartial
        if (not self._on_device(partial)
                or partial.dtype != torch.float32 or not partial.is_contiguous()
                or partial.numel() < 2 * n):
            raise ValueError(f"partial must be a contiguous float32 tensor on {self.device} with "
                             f">= {2 * n} elements ({n} records)")

    def _check_act(self, act: torch.Tensor, lead: tuple) -> torch.Tensor:
        shape = lead + (self.num_envs, 2)
        if act.shape != shape:
            raise AssertionError(f"actions shape {tuple(act.shape)} != {shape}")
        if act.dtype != torch.float32 or not self._on_device(act):
            raise TypeError(f"actions must be float32 on {self.device}")
        return act.contiguous()

    def step_tensor(self, actions: torch.Tensor, obs=None, rew=None, done=None):
        """One env step on device tensors; returns (obs [A,D], rew [A], done [A] bool)."""
        act = self._check_act(actions, ())
        obs = self.obs_dev if obs is None else obs
        rew = self.rew_dev if rew is None else rew
        done = self.done_dev if done is None else done
        A, D = self.num_envs, self.obs_dim
        self._check_out("obs", obs, (A, D), torch.float32)
        self._check_out("rew", rew, (A,), torch.float32)
        self._check_out("done", done, (A,), torch.bool)
        _lib.check(_lib.lib().fenv_step(self._h, _lib.ptr(act), _lib.ptr(obs), _lib.ptr(rew),
                                        _lib.ptr(done), self._stream()), "fenv_step")
        return obs, rew, done

    def rollout(self, actions: torch.Tensor, obs=None, rew=None, done=None, partial=None):
        """T fused env steps: actions [T, A, 2] -> obs [T, A, D], rew [T, A], done [T, A].

        Identical to T calls of :meth:`step_tensor`; state stays on chip for the whole launch."""
        T = int(actions.shape[0])
        act = self._check_act(actions, (T,))
        A, D, dev = self.num_envs, self.obs_dim, self.device
        if obs is None:
            obs = torch.empty((T, A, D), dtype=torch.float32, device=dev)
        if rew is None:
            rew = torch.empty((T, A), dtype=torch.float32, device=dev)
        if done is None:
            done = torch.empty((T, A), dtype=torch.bool, device=dev)
        self._check_out("obs", obs, (T, A, D), torch.float32)
        self._check_out("rew", rew, (T, A), torch.float32)
        self._check_out("done", done, (T, A), torch.bool)
        self._check_partial(partial)
        _lib.check(_lib.lib().fenv_rollout(self._h, T, _lib.ptr(act), _lib.ptr(obs),
                                           _lib.ptr(rew), _lib.ptr(done), _lib.ptr(partial),
                                           self._stream()), "fenv_rollout")
        return obs, rew, done

    def rollout_random(self, T: int, act_seed: int = 0, step_offset: int = 0, obs=None,
                       rew=None, done=None, partial=None, act_out=None):
        """Synthetic random-action rollout (``fenv_rollout_random``): T fused env steps whose
        U(-1, 1) actions are drawn inside the kernel from Philox keyed by ``act_seed``, counter
        (global agent, (step_offset + k) // 2).  ``act_out`` [T, A, 2] (optional) receives the
        actions; :meth:`rollout` on them from the same state returns the same bits."""
        T = int(T)
        if T < 0:
            raise ValueError("T must be >= 0")
        A, D, dev = self.num_envs, self.obs_dim, self.device
        if obs is None:
            obs = torch.empty((T, A, D), dtype=torch.float32, device=dev)
        if rew is None:
            rew = torch.empty((T, A), dtype=torch.float32, device=dev)
        if done is None:
            done = torch.empty((T, A), dtype=torch.bool, device=dev)
        self._check_out("act_out", act_out, (T, A, 2), torch.float32)
        self._check_out("obs", obs, (T, A, D), torch.float32)
        self._check_out("rew", rew, (T, A), torch.float32)
        self._check_out("done", done, (T, A), torch.bool)
        self._check_partial(partial)
        _lib.check(_lib.lib().fenv_rollout_random(
            self._h, T, int(act_seed) & 0xFFFFFFFFFFFFFFFF, int(step_offset) & 0xFFFFFFFFFFFFFFFF,
            _lib.ptr(act_out), _lib.ptr(obs), _lib.ptr(rew), _lib.ptr(done), _lib.ptr(partial),
            self._stream()), "fenv_rollout_random")
        return obs, rew, done

    def policy_rollout(self, params: torch.Tensor, T: int, bufs: dict, seed: int = 0,
                       offset: int = 0, deterministic: bool = False, gamma: float = 0.99,
                       gae_lambda: float = 0.95) -> None:
        """One fused launch (``fenv_policy_rollout``): T steps of policy forward (SB3 MlpPolicy
        on the flat ``params``) + env step, then the last value and GAE, written into the
        device tensors of ``bufs`` (keys = the fields of ``fenv_rollout_bufs``: obs, last_obs,
        mu, action, clipped, value, log_prob, reward, episode_start, done, last_done,
        last_value, advantage, ret; missing optional keys are skipped)."""
        if params.dtype != torch.float32 or params.device != self.device:
            raise TypeError(f"params must be float32 on {self.device}")
        n = int(_lib.lib().policy_param_count(self.obs_dim))
        if params.numel() != n or not params.is_contiguous():
            raise ValueError(f"params must be a contiguous float32 vector of {n} elements")
        T, A, D = int(T), self.num_envs, self.obs_dim
        f32, u8 = torch.float32, torch.bool
        shapes = dict(obs=((T, A, D), f32), last_obs=((A, D), f32), mu=((T, A, 2), f32),
                      action=((T, A, 2), f32), clipped=((T, A, 2), f32), value=((T, A), f32),
                      log_prob=((T, A), f32), reward=((T, A), f32),
                      episode_start=((T, A), u8), done=((T, A), u8), last_done=((A,), u8),
                      last_value=((A,), f32), advantage=((T, A), f32), ret=((T, A), f32))
        unknown = set(bufs) - set(shapes)
        if unknown:
            raise ValueError(f"unknown rollout buffers {sorted(unknown)}")
        rb = _lib.RolloutBufs()
        for name, _ in _lib.RolloutBufs._fields_:
            t = bufs.get(name)
            if t is not None:
                shp, dt = shapes[name]
                self._check_out(name, t, shp, dt)
                setattr(rb, name, t.data_ptr())
        _lib.check(_lib.lib().fenv_policy_rollout(
            self._h, _lib.ptr(params), int(T), int(seed) & 0xFFFFFFFFFFFFFFFF, int(offset),
            int(bool(deterministic)), float(gamma), float(gae_lambda), ctypes.byref(rb),
            self._stream()), "fenv_policy_rollout")

    def partial_count(self) -> int:
        return int(_lib.lib().fenv_partial_count(self._h))

    def reduce_partials(self, partial: torch.Tensor, out: torch.Tensor | None = None):
        """Sum the per-wavefront {reward, done} records of :meth:`rollout` -> double[2]."""
        self._check_partial(partial)
        if out is None:
            out = torch.empty(2, dtype=torch.float64, device=self.device)
        self._check_out("out", out, (2,), torch.float64)
        _lib.check(_lib.lib().fenv_reduce_partials(_lib.ptr(partial), self.partial_count(),
                                                   _lib.ptr(out), self._stream()),
                   "fenv_reduce_partials")
        return out

    METRIC_NAMES = ("avg_dist_to_goal", "ave_dist_to_neighbor", "std_dist_to_neighbor", "reward",
                    "close_to_goal_reward", "reward_dist", "reward_right_neighbor",
                    "reward_left_neighbor")

    def rollout_kernel_name(self, T: int) -> str:
        """The kernel fenv_rollout launches for a T-step launch of this env (diagnostic)."""
        return _lib.lib().fenv_rollout_kernel(self._h, int(T)).decode()

    def metrics(self, rew: torch.Tensor | None = None, sums: torch.Tensor | None = None):
        """Per-formation wandb statistics of the reference, device tensor [F, 8] (columns
        METRIC_NAMES): compute_metrics (simulate.py:238-254) on the current state, the mean
        reward (vectorized_env.py:80-81), and the means of compute_reward_and_done's logged
        components (simulate.py:183-208) for the state the latest step scored.  ``sums``
        (float64 [8], optional) receives the column sums over formations."""
        self._check_out("rew", rew, (self.num_envs,), torch.float32)
        self._check_out("sums", sums, (8,), torch.float64)
        out = torch.empty((self.num_formation, 8), dtype=torch.float32, device=self.device)
        _lib.check(_lib.lib().fenv_metrics(self._h, _lib.ptr(rew), _lib.ptr(out), _lib.ptr(sums),
                                           self._stream()), "fenv_metrics")
        return out

    def get_state(self):
        """(px [A], py [A], gx [F], gy [F], steps_since_reset [F]) as device tensors."""
        A, F, dev = self.num_envs, self.num_formation, self.device
        px = torch.empty(A, dtype=torch.float32, device=dev)
        py = torch.empty(A, dtype=torch.float32, device=dev)
        gx = torch.empty(F, dtype=torch.float32, device=dev)
        gy = torch.empty(F, dtype=torch.float32, device=dev)
        t = torch.empty(F, dtype=torch.int32, device=dev)
        _lib.check(_lib.lib().fenv_get_state(self._h, *(_lib.ptr(v) for v in (px, py, gx, gy, t)),
                                             self._stream()), "fenv_get_state")
        return px, py, gx, gy, t

    def _check_range(self, first: int, count: int) -> tuple:
        first, count = int(first), int(count)
        if count < 1 or first < 0 or first + count > self.num_formation:
            raise IndexError(f"formations [{first}, {first + count}) outside [0, "
                             f"{self.num_formation})")
        return first, count

    def get_state_range(self, first: int, count: int):
        """State of formations [first, first + count) only (``fenv_get_state_range``):
        (px [count*N], py [count*N], gx [count], gy [count], t [count]) device tensors."""
        first, count = self._check_range(first, count)
        n, dev = count * self.num_agents_per_formation, self.device
        px = torch.empty(n, dtype=torch.float32, device=dev)
        py = torch.empty(n, dtype=torch.float32, device=dev)
        gx = torch.empty(count, dtype=torch.float32, device=dev)
        gy = torch.empty(count, dtype=torch.float32, device=dev)
        t = torch.empty(count, dtype=torch.int32, device=dev)
        _lib.check(_lib.lib().fenv_get_state_range(
            self._h, first, count, *(_lib.ptr(v) for v in (px, py, gx, gy, t)), self._stream()),
            "fenv_get_state_range")
        return px, py, gx, gy, t

    def metrics_range(self, first: int, count: int, rew: torch.Tensor | None = None):
        """:meth:`metrics` of formations [first, first + count) only (``fenv_metrics_range``):
        [count, 8]; ``rew`` (optional) holds those formations' count*N rewards."""
        first, count = self._check_range(first, count)
        self._check_out("rew", rew, (count * self.num_agents_per_formation,), torch.float32)
        out = torch.empty((count, 8), dtype=torch.float32, device=self.device)
        _lib.check(_lib.lib().fenv_metrics_range(self._h, first, count, _lib.ptr(rew),
                                                 _lib.ptr(out), None, self._stream()),
                   "fenv_metrics_range")
        return out

    def set_state(self, px, py, gx, gy, t) -> None:
        dev = self.device
        vals = [torch.as_tensor(v, dtype=torch.float32).to(dev).contiguous()
                for v in (px, py, gx, gy)]
        tt = torch.as_tensor(t, dtype=torch.int32).to(dev).contiguous()
        A, F = self.num_envs, self.num_formation
        for v, n in zip(vals, (A, A, F, F)):
            if v.numel() != n:
                raise ValueError("set_state: wrong sizes")
        if tt.numel() != F:
            raise ValueError("set_state: wrong sizes")
        _lib.check(_lib.lib().fenv_set_state(self._h, *(_lib.ptr(v) for v in vals), _lib.ptr(tt),
                                             self._stream()), "fenv_set_state")
