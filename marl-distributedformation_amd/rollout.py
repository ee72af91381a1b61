"""Device-resident rollout collection (SB3 ``collect_rollouts`` + ``RolloutBuffer``) for PPO.

The reference trains with ``PPO('MlpPolicy', env, n_steps=10, ...)`` (vectorized_env.py:126-134):
every env step SB3 moves obs to the policy device, samples actions, clips them to the Box,
calls ``env.step`` on numpy arrays and appends to host numpy buffers ``[n_steps, n_envs, .]``.
Here the whole loop stays in HBM: :class:`RolloutBuffer` holds ``[T, A, .]`` device tensors, the
policy forward (``policy_forward``) writes actions/values/log-probs straight into them, the env
step (``fenv_step``) writes rewards/dones, and GAE runs in one kernel (``rollout_gae``).
Semantics follow SB3 2.x ``OnPolicyAlgorithm.collect_rollouts`` / ``RolloutBuffer``: the buffer
stores the obs the action was taken on, the UNCLIPPED action, ``episode_starts`` = the previous
step's dones, and no timeout bootstrap (the reference's infos carry no ``TimeLimit`` keys).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from . import _lib


@dataclass
class RolloutBatch:
    observations: torch.Tensor
    actions: torch.Tensor
    old_values: torch.Tensor
    old_log_prob: torch.Tensor
    advantages: torch.Tensor
    returns: torch.Tensor


class RolloutBuffer:
    """``[T, A, .]`` device buffers (SB3 RolloutBuffer fields)."""

    def __init__(self, n_steps: int, n_envs: int, obs_dim: int, device, gamma: float = 0.99,
                 gae_lambda: float = 0.95):
        T, A, dev = int(n_steps), int(n_envs), torch.device(device)
        self.n_steps, self.n_envs, self.obs_dim, self.device = T, A, obs_dim, dev
        self.gamma, self.gae_lambda = float(gamma), float(gae_lambda)
        f32 = dict(dtype=torch.float32, device=dev)
        self.observations = torch.zeros((T, A, obs_dim), **f32)
        self.actions = torch.zeros((T, A, 2), **f32)
        self.clipped = torch.zeros((T, A, 2), **f32)
        self.rewards = torch.zeros((T, A), **f32)
        self.values = torch.zeros((T, A), **f32)
        self.log_probs = torch.zeros((T, A), **f32)
        self.mu = torch.zeros((T, A, 2), **f32)
        self.episode_starts = torch.zeros((T, A), dtype=torch.bool, device=dev)
        self.dones = torch.zeros((T, A), dtype=torch.bool, device=dev)
        self.advantages = torch.zeros((T, A), **f32)
        self.returns = torch.zeros((T, A), **f32)
        self.pos = 0

    def reset(self) -> None:
        self.pos = 0

    def full(self) -> bool:
        return self.pos == self.n_steps

    def compute_returns_and_advantage(self, last_values: torch.Tensor,
                                      dones: torch.Tensor) -> None:
        """SB3 RolloutBuffer.compute_returns_and_advantage (GAE), one HIP kernel."""
        lv = last_values.contiguous().float()
        ld = dones.contiguous().to(torch.bool)
        _lib.check(_lib.lib().rollout_gae(
            _lib.ptr(self.rewards), _lib.ptr(self.values), _lib.ptr(self.episode_starts),
            _lib.ptr(lv), _lib.ptr(ld), self.n_steps, self.n_envs, self.gamma, self.gae_lambda,
            _lib.ptr(self.advantages), _lib.ptr(self.returns), _lib.current_stream(self.device)),
            "rollout_gae")

    def get(self, batch_size: int | None, generator: torch.Generator | None = None):
        """Shuffled minibatches over the flattened T*A samples (SB3 RolloutBuffer.get)."""
        n = self.n_steps * self.n_envs
        idx = torch.randperm(n, device=self.device, generator=generator)
        bs = n if batch_size is None else int(batch_size)
        obs = self.observations.reshape(n, self.obs_dim)
        act = self.actions.reshape(n, 2)
        val = self.values.reshape(n)
        lp = self.log_probs.reshape(n)
        adv = self.advantages.reshape(n)
        ret = self.returns.reshape(n)
        for s in range(0, n, bs):
            j = idx[s:s + bs]
            yield RolloutBatch(obs[j], act[j], val[j], lp[j], adv[j], ret[j])


class RolloutCollector:
    """SB3 ``collect_rollouts`` on device.

    ``fused=True`` (default whenever the formation fits a wavefront, N <= 64) runs the whole
    rollout -- T x (policy forward + env step), last value, GAE -- as ONE kernel
    (``fenv_policy_rollout``); ``fused=False`` issues policy_forward + fenv_step per step and a
    GAE launch.  Both produce identical bits (tests/test_gpu_rollout.py)."""

    def __init__(self, env, policy, buffer: RolloutBuffer, seed: int = 0,
                 fused: bool | None = None):
        if buffer.n_envs != env.num_envs or buffer.obs_dim != env.obs_dim:
            raise ValueError("buffer shape does not match the env")
        self.env, self.policy, self.buffer = env, policy, buffer
        self.fused = env.num_agents_per_formation <= 64 if fused is None else bool(fused)
        self.seed = int(seed)
        self.offset = 0
        self.num_timesteps = 0
        self.last_obs = env.reset_tensor().clone()
        self.last_episode_starts = torch.ones(env.num_envs, dtype=torch.bool, device=env.device)
        # torch.bool is one byte per element: the kernels read/write it as uint8
        self._last_values = torch.empty(env.num_envs, dtype=torch.float32, device=env.device)

    def collect(self, deterministic: bool = False) -> RolloutBuffer:
        if self.fused:
            return self._collect_fused(deterministic)
        return self._collect_steps(deterministic)

    def _collect_fused(self, deterministic: bool) -> RolloutBuffer:
        b = self.buffer
        b.reset()
        T = b.n_steps
        self.env.policy_rollout(
            self.policy.flat, T, dict(
                obs=b.observations, last_obs=self.last_obs, mu=b.mu, action=b.actions,
                clipped=b.clipped, value=b.values, log_prob=b.log_probs, reward=b.rewards,
                episode_start=b.episode_starts, done=b.dones,
                last_done=self.last_episode_starts, last_value=self._last_values,
                advantage=b.advantages, ret=b.returns),
            seed=self.seed, offset=self.offset, deterministic=deterministic, gamma=b.gamma,
            gae_lambda=b.gae_lambda)
        self.offset += T
        self.num_timesteps += T * self.env.num_envs
        b.pos = T
        return b

    def _collect_steps(self, deterministic: bool) -> RolloutBuffer:
        """n_steps x (policy_forward + fenv_step), two launches per step and no copies: the env
        writes step k's observation straight into observations[k+1] and its dones into
        episode_starts[k+1] (SB3's episode_starts are the previous step's dones)."""
        b = self.buffer
        b.reset()
        T = b.n_steps
        b.observations[0].copy_(self.last_obs)
        b.episode_starts[0].copy_(self.last_episode_starts)
        row0 = self.env.first_formation * self.env.num_agents_per_formation  # global noise rows
        for k in range(T):
            self.policy.forward(b.observations[k], deterministic=deterministic,
                                out=dict(mu=b.mu[k], value=b.values[k], action=b.actions[k],
                                         log_prob=b.log_probs[k], clipped=b.clipped[k]),
                                seed=self.seed, offset=self.offset, row0=row0)
            self.offset += 1
            last = k == T - 1
            # the env is stepped with the clipped action (collect_rollouts np.clip)
            self.env.step_tensor(b.clipped[k],
                                 obs=self.last_obs if last else b.observations[k + 1],
                                 rew=b.rewards[k],
                                 done=self.last_episode_starts if last else b.episode_starts[k + 1])
            self.num_timesteps += self.env.num_envs
            b.pos += 1
        b.dones[:-1].copy_(b.episode_starts[1:])
        b.dones[-1].copy_(self.last_episode_starts)
        self.policy.forward(self.last_obs, deterministic=True, out=dict(value=self._last_values),
                            seed=self.seed, offset=0)  # value of the final observation
        b.compute_returns_and_advantage(self._last_values, self.last_episode_starts)
        return b
