"""PPO update on device, SB3 2.x ``PPO.train`` semantics, PyTorch-ROCm autograd.

The reference's training run (vectorized_env.py:126-137) is SB3 PPO with ``n_steps=10``,
``learning_rate=1e-3``, ``ent_coef=0.01`` and SB3 defaults otherwise (``n_epochs=10``,
``batch_size=64``, ``gamma=0.99``, ``gae_lambda=0.95``, ``clip_range=0.2``, ``vf_coef=0.5``,
``max_grad_norm=0.5``, advantage normalisation, Adam eps 1e-5).  Rollouts come from
:class:`rollout.RolloutCollector` (HIP kernels); the update differentiates a torch restatement of
the same MLP over the SAME flat parameter buffer the kernel reads, so the gradient is one
contiguous 9,669-float bucket: with several ranks it is all-reduced once per optimizer step
(RCCL over xGMI), never per tensor.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.distributed as dist
import torch.nn.functional as Fn

from . import checkpoint as ckpt
from .policy import MlpPolicy
from .rollout import RolloutBuffer, RolloutCollector


@dataclass
class PPOConfig:
    n_steps: int = 10            # vectorized_env.py:128
    learning_rate: float = 1e-3  # vectorized_env.py:130
    ent_coef: float = 0.01       # vectorized_env.py:131
    n_epochs: int = 10           # SB3 defaults below
    batch_size: int = 64
    gamma: float = 0.99
    gae_lambda: float = 0.95
    clip_range: float = 0.2
    vf_coef: float = 0.5
    max_grad_norm: float = 0.5
    normalize_advantage: bool = True


def evaluate_actions(policy: MlpPolicy, flat: torch.Tensor, obs: torch.Tensor,
                     actions: torch.Tensor):
    """SB3 ActorCriticPolicy.evaluate_actions as differentiable torch ops on views of `flat`."""
    D = policy.obs_dim
    o = 0
    P = {}
    for k, shp in policy.param_shapes():
        n = math.prod(shp)
        P[k] = flat[o:o + n].view(shp)
        o += n
    h = torch.tanh(Fn.linear(obs, P["mlp_extractor.policy_net.0.weight"],
                             P["mlp_extractor.policy_net.0.bias"]))
    h = torch.tanh(Fn.linear(h, P["mlp_extractor.policy_net.2.weight"],
                             P["mlp_extractor.policy_net.2.bias"]))
    v = torch.tanh(Fn.linear(obs, P["mlp_extractor.value_net.0.weight"],
                             P["mlp_extractor.value_net.0.bias"]))
    v = torch.tanh(Fn.linear(v, P["mlp_extractor.value_net.2.weight"],
                             P["mlp_extractor.value_net.2.bias"]))
    mu = Fn.linear(h, P["action_net.weight"], P["action_net.bias"])
    values = Fn.linear(v, P["value_net.weight"], P["value_net.bias"]).squeeze(-1)
    log_std = P["log_std"]
    std = log_std.exp().expand_as(mu)
    var = std * std
    log_prob = (-((actions - mu) ** 2) / (2 * var) - std.log()
                - math.log(math.sqrt(2 * math.pi))).sum(-1)
    entropy = (0.5 + 0.5 * math.log(2 * math.pi) + std.log()).sum(-1)
    del D
    return values, log_prob, entropy


class PPO:
    """Minimal on-device PPO: collect (HIP kernels) -> GAE (HIP) -> clipped-surrogate update."""

    def __init__(self, env, cfg: PPOConfig | None = None, seed: int = 0, policy=None):
        self.cfg = cfg or PPOConfig()
        self.seed = int(seed)
        self.env = env
        self.policy = policy or MlpPolicy(env.obs_dim, device=env.device, seed=seed)
        self.buffer = RolloutBuffer(self.cfg.n_steps, env.num_envs, env.obs_dim, env.device,
                                    self.cfg.gamma, self.cfg.gae_lambda)
        self.collector = RolloutCollector(env, self.policy, self.buffer, seed=seed)
        self.param = torch.nn.Parameter(self.policy.flat)  # shares storage with the kernel's
        self.opt = torch.optim.Adam([self.param], lr=self.cfg.learning_rate, eps=1e-5)
        self.gen = torch.Generator(device=env.device).manual_seed(seed)
        self.world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        self.stats: dict = {}

    @property
    def num_timesteps(self) -> int:
        return self.collector.num_timesteps * self.world

    def train(self) -> dict:
        c = self.cfg
        pg, vl, el, cf, n = 0.0, 0.0, 0.0, 0.0, 0
        for _ in range(c.n_epochs):
            for b in self.buffer.get(c.batch_size, self.gen):
                values, log_prob, entropy = evaluate_actions(self.policy, self.param,
                                                             b.observations, b.actions)
                adv = b.advantages
                if c.normalize_advantage and adv.numel() > 1:
                    adv = (adv - adv.mean()) / (adv.std() + 1e-8)
                ratio = torch.exp(log_prob - b.old_log_prob)
                l1 = adv * ratio
                l2 = adv * torch.clamp(ratio, 1 - c.clip_range, 1 + c.clip_range)
                policy_loss = -torch.min(l1, l2).mean()
                value_loss = Fn.mse_loss(b.returns, values)
                entropy_loss = -torch.mean(entropy)
                loss = policy_loss + c.ent_coef * entropy_loss + c.vf_coef * value_loss
                self.opt.zero_grad(set_to_none=False)
                loss.backward()
                if self.world > 1:  # one flat bucket per optimizer step
                    dist.all_reduce(self.param.grad)
                    self.param.grad.div_(self.world)
                torch.nn.utils.clip_grad_norm_([self.param], c.max_grad_norm)
                self.opt.step()
                pg += float(policy_loss.detach())
                vl += float(value_loss.detach())
                el += float(entropy_loss.detach())
                cf += float((torch.abs(ratio - 1) > c.clip_range).float().mean())
                n += 1
        self.stats = dict(policy_gradient_loss=pg / n, value_loss=vl / n, entropy_loss=el / n,
                          clip_fraction=cf / n)
        return self.stats

    def learn(self, total_timesteps: int, callback=None) -> "PPO":
        """SB3 ``learn``: alternate collect_rollouts and train until total_timesteps.

        ``callback`` is a :class:`checkpoint.CheckpointCallback` (run after each collection, as
        SB3 runs its ``_on_step`` inside ``collect_rollouts``; only rank 0 writes), a plain
        function ``f(ppo)`` called after each train (returning False stops), or a list of both."""
        cbs = callback if isinstance(callback, (list, tuple)) else [callback]
        rank = dist.get_rank() if self.world > 1 else 0
        while self.num_timesteps < total_timesteps:
            with torch.no_grad():
                self.collector.collect()
            for cb in cbs:
                if hasattr(cb, "on_steps") and rank == 0:
                    cb.on_steps(self, self.cfg.n_steps, self.env.num_envs * self.world)
            self.train()
            stop = False
            for cb in cbs:
                if cb is not None and not hasattr(cb, "on_steps") and cb(self) is False:
                    stop = True
            if stop:
                break
        return self

    # ---------------------------------------------------------------- SB3 model zips
    def hyperparameters(self) -> dict:
        c = self.cfg
        return {"n_steps": c.n_steps, "learning_rate": c.learning_rate, "ent_coef": c.ent_coef,
                "n_epochs": c.n_epochs, "batch_size": c.batch_size, "gamma": c.gamma,
                "gae_lambda": c.gae_lambda, "clip_range": c.clip_range, "vf_coef": c.vf_coef,
                "max_grad_norm": c.max_grad_norm, "normalize_advantage": c.normalize_advantage,
                "n_envs": self.env.num_envs * self.world, "seed": self.seed}

    def save(self, path: str, num_timesteps: int | None = None) -> str:
        """SB3 ``model.save(path)``: an SB3-layout zip (checkpoint.py) with the policy's SB3
        state_dict, the Adam state re-expressed per SB3 tensor, and the hyper-parameters."""
        t = self.num_timesteps if num_timesteps is None else int(num_timesteps)
        opt = ckpt.optimizer_state_from_flat(self.policy.param_shapes(), self.opt.state_dict())
        return ckpt.save_sb3_zip(path, self.policy.state_dict(), num_timesteps=t,
                                 data=self.hyperparameters(), optimizer_state=opt)

    @classmethod
    def load(cls, path: str, env, cfg: PPOConfig | None = None, seed: int = 0) -> "PPO":
        """SB3 ``PPO.load(path, env)``: hyper-parameters from the zip's ``data`` (unless ``cfg``
        is given), policy weights from its ``policy.pth``."""
        sd, data = ckpt.load_sb3_zip(path)
        if cfg is None:
            fields = PPOConfig.__dataclass_fields__
            cfg = PPOConfig(**{k: data[k] for k in fields if k in data})
        model = cls(env, cfg, seed=seed)
        model.policy.load_state_dict(sd)
        model.loaded_num_timesteps = int(data.get("num_timesteps", 0))
        return model
