"""Per-formation views over the device-resident env (the reference's FormationSimulator face).

The reference keeps one ``FormationSimulator`` object per formation (simulate.py:7-254) and
exposes them as ``FormationEnv.formationsim_list`` (vectorized_env.py:38-43); its consumers read
``agents``, ``goal``, ``steps_since_reset`` and, for formation 0 in playback, the matplotlib
``fig`` (visualize_policy.py:38,43).  Here the state of every formation lives in HBM inside one
libfenv handle, so ``formationsim_list`` is a lazy sequence of read-only views.  A view reads
only its own formation: ``fenv_get_state_range`` copies its N agents' slice and
``fenv_metrics_range`` scores only that formation, so one access costs O(N), whatever the env's
size.  The simulation itself never runs through them.

Views hold the env through a weak reference: an env and its views form no reference cycle, so a
dropped env is freed by reference counting at a known point rather than by the cyclic garbage
collector at an arbitrary one.
"""
from __future__ import annotations

import weakref
from collections.abc import Sequence

import numpy as np
import torch


class FormationView:
    """Read-only host view of formation ``index`` (simulate.py:7 FormationSimulator fields)."""

    width = 400       # simulate.py:13
    height = 600      # simulate.py:14
    max_steps = 1000  # simulate.py:20 (the env's value is authoritative)
    desired_radius = 60
    obstacle_size = 10
    num_obstacles = 0

    def __init__(self, env, index: int):
        self._envref = weakref.ref(env)
        self.index = int(index)
        self.num_agents = env.num_agents_per_formation
        self.goal_in_obs = env.goal_in_obs
        self.share_reward_ratio = env.share_reward_ratio
        self.desired_neighbor_dist = float(env.desired_neighbor_dist)
        self.visualize = False
        self.log = False

    @property
    def _env(self):
        env = self._envref()
        if env is None:
            raise ReferenceError("the FormationEnv of this view no longer exists")
        return env

    # -- state (simulate.py:133 agents [N,2], :140 goal [2], :147 steps_since_reset)
    def _slice(self):
        return self._env._formation_state(self.index)

    @property
    def agents(self) -> torch.Tensor:
        px, py, _, _, _ = self._slice()
        return torch.from_numpy(np.stack([px, py], axis=1))

    @property
    def goal(self) -> torch.Tensor:
        _, _, gx, gy, _ = self._slice()
        return torch.tensor([gx, gy], dtype=torch.float32)

    @property
    def steps_since_reset(self) -> int:
        return int(self._slice()[4])

    @property
    def obstacles(self) -> torch.Tensor:
        return torch.zeros((0, 2))

    def compute_obs(self) -> torch.Tensor:
        """Observation rows of this formation (simulate.py:150-174)."""
        env = self._env
        obs = env.observe_tensor()
        N = self.num_agents
        return obs[self.index * N:(self.index + 1) * N].cpu()

    def _metrics(self) -> list:
        return self._env.metrics_range(self.index, 1)[0].tolist()

    def compute_metrics(self) -> dict:
        """simulate.py:238-254 (the values the reference logs when ``log``)."""
        m = self._metrics()
        return {"avg_dist_to_goal": m[0], "ave_dist_to_neighbor": m[1],
                "std_dist_to_neighbor": m[2]}

    def reward_components(self) -> dict:
        """The means compute_reward_and_done logs (simulate.py:183-208) for the last step."""
        m = self._metrics()
        return dict(zip(("close_to_goal_reward", "reward_dist", "reward_right_neighbor",
                         "reward_left_neighbor"), m[4:8]))

    def __repr__(self) -> str:
        return f"FormationView(index={self.index}, num_agents={self.num_agents})"


class FormationViewList(Sequence):
    """Lazy ``formationsim_list``: view objects are created on first access and cached."""

    def __init__(self, env, count: int):
        self._envref = weakref.ref(env)
        self._n = int(count)
        self._cache: dict[int, FormationView] = {}

    def __len__(self) -> int:
        return self._n

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(self._n))]
        i = int(i)
        if i < 0:
            i += self._n
        if not 0 <= i < self._n:
            raise IndexError("formation index out of range")
        v = self._cache.get(i)
        if v is None:
            env = self._envref()
            if env is None:
                raise ReferenceError("the FormationEnv of this list no longer exists")
            v = self._cache[i] = env._make_view(i)
        return v
