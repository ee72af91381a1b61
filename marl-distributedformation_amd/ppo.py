"""PPO update on device, SB3 2.x ``PPO.train`` semantics, PyTorch-ROCm autograd.

The reference's training run (vectorized_env.py:126-137) is SB3 PPO with ``n_steps=10``,
``learning_rate=1e-3``, ``ent_coef=0.01`` and SB3 defaults otherwise (``n_epochs=10``,
``batch_size=64``, ``gamma=0.99``, ``gae_lambda=0.95``, ``clip_range=0.2``, ``vf_coef=0.5``,
``max_grad_norm=0.5``, advantage normalisation, Adam eps 1e-5).  Rollouts come from
:class:`rollout.RolloutCollector` (HIP kernels); the update differentiates a torch restatement of
the same MLP over the SAME flat parameter buffer the kernel reads.

Several ranks (one process per GPU, formations sharded): every rank collects its shard's rollout
(policy noise keyed by the GLOBAL agent index, so the shards together draw exactly what the
unsharded env draws), then ONE all-gather per update assembles the global [T, A_total] sample
buffer in the unsharded order, and every rank runs the same update on it with the same
permutations -- parameters and Adam state stay bitwise identical with no per-minibatch
collective, and the result is the single-process update of the unsharded buffer.
"""
from __future__ import annotations

import ctypes
import gc
import math
import warnings
from dataclasses import dataclass

import torch
import torch.distributed as dist
import torch.nn.functional as Fn

from . import checkpoint as ckpt
from . import distributed as pdist
from .dp_update import ShardedUpdate
from .policy import MlpPolicy, param_shapes
from .rollout import RolloutBuffer, RolloutCollector

_CAPTURE_STREAMS: dict = {}


def _capture_stream(device: torch.device) -> torch.cuda.Stream:
    """One capture stream per device for every PPO instance of the process: a fresh stream per
    capture made the 8th capture in one process fail inside hipBLASLt
    (tools/graph_capture_probe.py)."""
    key = torch.device(device).index
    if key not in _CAPTURE_STREAMS:
        _CAPTURE_STREAMS[key] = torch.cuda.Stream(device)
    return _CAPTURE_STREAMS[key]


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
    # several ranks: "replicated" = one all-gather of every rank's samples per update, then the
    # same sequential update on every rank (SB3's exact minibatches); "sharded" = each rank keeps
    # its samples and takes batch_size / world rows of every global minibatch, with one gradient
    # all-reduce per minibatch (dp_update.py)
    update_mode: str = "replicated"


def evaluate_actions(policy, flat: torch.Tensor, obs: torch.Tensor, actions: torch.Tensor):
    """SB3 ActorCriticPolicy.evaluate_actions as differentiable torch ops on views of `flat`.
    ``policy``: an :class:`MlpPolicy`, or the observation size (int) alone."""
    shapes = param_shapes(policy) if isinstance(policy, int) else policy.param_shapes()
    o = 0
    P = {}
    for k, shp in shapes:
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
    return values, log_prob, entropy


def epoch_permutations(n: int, n_epochs: int, gen: torch.Generator, device) -> torch.Tensor:
    """[n_epochs, n] int64: one ``torch.randperm(n)`` per epoch from ``gen`` (SB3's
    RolloutBuffer.get draws one permutation per epoch)."""
    perm = torch.empty((int(n_epochs), int(n)), dtype=torch.long, device=device)
    for e in range(int(n_epochs)):
        perm[e].copy_(torch.randperm(int(n), device=device, generator=gen))
    return perm


class PPO:
    """Minimal on-device PPO: collect (HIP kernels) -> GAE (HIP) -> clipped-surrogate update."""

    def __init__(self, env, cfg: PPOConfig | None = None, seed: int = 0, policy=None,
                 use_graph: bool | None = None, use_fused: bool | None = None):
        self.cfg = cfg or PPOConfig()
        self.seed = int(seed)
        self.env = env
        self.policy = policy or MlpPolicy(env.obs_dim, device=env.device, seed=seed)
        self.buffer = RolloutBuffer(self.cfg.n_steps, env.num_envs, env.obs_dim, env.device,
                                    self.cfg.gamma, self.cfg.gae_lambda)
        self.world, self.rank = pdist.world_rank()
        # replicated weights: rank 0's, once (a loaded checkpoint or seed-identical init alike);
        # one noise seed for all ranks (the kernels key the noise by global agent index)
        pdist.broadcast_(self.policy.flat)
        self.collector = RolloutCollector(env, self.policy, self.buffer, seed=seed)
        N = env.num_agents_per_formation
        self.total_envs = env.num_envs
        self.counts = [env.num_envs]
        if self.world > 1:  # the env is this rank's shard of total_formations
            self.total_envs = int(env.total_formations) * N
            self.counts = pdist.shard_counts(int(env.total_formations), self.world, N)
            if self.counts[self.rank] != env.num_envs:
                raise ValueError("env shard does not match distributed.shard_range(total_formations, "
                                 "rank, world)")
        if self.cfg.update_mode not in ("replicated", "sharded"):
            raise ValueError("update_mode must be 'replicated' or 'sharded'")
        self.sharded = self.cfg.update_mode == "sharded"
        T, D = self.cfg.n_steps, env.obs_dim
        # update samples [T, A_total, D + 5] = obs | action(2) | log_prob | advantage | return;
        # with one rank (or the sharded update) they are views of the rollout buffer instead
        rep_gather = self.world > 1 and not self.sharded
        self._gsamples = (torch.empty((T, self.total_envs, D + 5), dtype=torch.float32,
                                      device=env.device) if rep_gather else None)
        self._lsamples = (torch.empty((T, env.num_envs, D + 5), dtype=torch.float32,
                                      device=env.device) if rep_gather else None)
        self.param = torch.nn.Parameter(self.policy.flat)  # shares storage with the kernel's
        self.param.grad = torch.zeros_like(self.param)     # static: graph replays write it
        # capturable: the step count lives on the device, so the update can be graph-captured
        self.opt = torch.optim.Adam([self.param], lr=self.cfg.learning_rate, eps=1e-5,
                                    capturable=True)
        self.gen = torch.Generator(device=env.device).manual_seed(seed)
        self.stats: dict = {}
        # minibatch update as HIP graphs (one replay per minibatch instead of ~60 launches)
        self.use_graph = (self.param.device.type == "cuda") if use_graph is None else use_graph
        n = self.buffer.n_steps * self.total_envs
        dev = self.param.device
        self._perm = torch.zeros(n, dtype=torch.long, device=dev)
        self._k = torch.zeros((), dtype=torch.long, device=dev)
        self._sums = torch.zeros(4, dtype=torch.float64, device=dev)
        self.exchange_retries = 0  # fused update launches re-run after a lost norm exchange
        self._graphs = None
        # batch_size <= 64 (SB3's default 64): the whole update as one HIP kernel (ppo_update)
        self.use_fused = ((self.param.device.type == "cuda" and self.cfg.batch_size <= 64)
                          if use_fused is None else use_fused)
        # the fused update's exchange words: this instance's own (include/fenv.h ppo_update_ws)
        from . import _lib
        self._ws = (torch.zeros(int(_lib.lib().ppo_workspace_bytes()), dtype=torch.uint8,
                                device=dev) if self.param.device.type == "cuda" else None)
        self._dp = None
        if self.sharded:
            # one rank: the replicated path's generator, so both modes draw the same minibatches
            self._dp = ShardedUpdate(self.cfg, D, [T * c for c in self.counts], seed, dev,
                                     fused=self.use_fused,
                                     gen=self.gen if self.world == 1 else None)
            if self.world > 1:
                warnings.warn("PPOConfig(update_mode='sharded'): each rank shuffles its own "
                              "samples, so the minibatch sequence (and the training trajectory) "
                              "is not SB3's; update_mode='replicated' reproduces SB3's update "
                              "exactly", RuntimeWarning, stacklevel=2)

    @property
    def num_timesteps(self) -> int:
        """Env steps of ALL ranks' agents so far (identical on every rank)."""
        return self.collector.num_timesteps // self.env.num_envs * self.total_envs

    # ---------------------------------------------------------------- samples
    def gather_samples(self) -> None:
        """World > 1: assemble the global update buffer (one all-gather, unsharded order)."""
        if self.world == 1 or self.sharded:
            return
        b, D = self.buffer, self.buffer.obs_dim
        ls = self._lsamples
        ls[..., :D].copy_(b.observations)
        ls[..., D:D + 2].copy_(b.actions)
        ls[..., D + 2].copy_(b.log_probs)
        ls[..., D + 3].copy_(b.advantages)
        ls[..., D + 4].copy_(b.returns)
        pdist.gather_columns(ls, self.counts, out=self._gsamples)

    def _flat(self):
        """(obs, actions, old_log_prob, advantages, returns) over the update's n samples."""
        b, D = self.buffer, self.buffer.obs_dim
        if self.world == 1 or self.sharded:
            n = b.n_steps * b.n_envs
            return (b.observations.reshape(n, D), b.actions.reshape(n, 2),
                    b.log_probs.reshape(n), b.advantages.reshape(n), b.returns.reshape(n))
        g = self._gsamples
        n = g.shape[0] * g.shape[1]
        g2 = g.view(n, D + 5)
        return g2[:, :D], g2[:, D:D + 2], g2[:, D + 2], g2[:, D + 3], g2[:, D + 4]

    def _permutations(self, n: int) -> torch.Tensor:
        """SB3 RolloutBuffer.get's randperm, one per epoch, from this PPO's generator (seeded
        alike on every rank, so all ranks draw the same permutations)."""
        return epoch_permutations(n, self.cfg.n_epochs, self.gen, self.param.device)

    # ---------------------------------------------------------------- one minibatch

    def _forward_backward(self, idx: torch.Tensor) -> None:
        """SB3 PPO.train inner loop up to loss.backward() for minibatch ``idx``; adds the
        minibatch's (policy loss, value loss, entropy loss, clip fraction) to self._sums."""
        c = self.cfg
        obs, act, old_lp, adv, ret = (t[idx] for t in self._flat())
        values, log_prob, entropy = evaluate_actions(self.policy, self.param, obs, act)
        if c.normalize_advantage and adv.numel() > 1:
            adv = (adv - adv.mean()) / (adv.std() + 1e-8)
        ratio = torch.exp(log_prob - old_lp)
        l1 = adv * ratio
        l2 = adv * torch.clamp(ratio, 1 - c.clip_range, 1 + c.clip_range)
        policy_loss = -torch.min(l1, l2).mean()
        value_loss = Fn.mse_loss(ret, values)
        entropy_loss = -torch.mean(entropy)
        loss = policy_loss + c.ent_coef * entropy_loss + c.vf_coef * value_loss
        self.param.grad.zero_()
        loss.backward()
        clip_fraction = (torch.abs(ratio - 1) > c.clip_range).float().mean()
        self._sums += torch.stack([policy_loss.detach(), value_loss.detach(),
                                   entropy_loss.detach(), clip_fraction]).double()

    def _apply(self) -> None:
        torch.nn.utils.clip_grad_norm_([self.param], self.cfg.max_grad_norm)
        self.opt.step()

    def _eager_step(self, idx: torch.Tensor) -> None:
        self._forward_backward(idx)
        self._apply()

    def _capture(self, warm_idx: list) -> None:
        """Record the full-minibatch step as one HIP graph: gather + forward + backward + stats,
        k += 1, clip + Adam.  The warm-up runs the first real minibatches eagerly on the capture
        stream."""
        bs = self.cfg.batch_size
        # every tensor the graphs read must outlive them (a freed one's memory gets reused and
        # the replay would gather with garbage indices): attributes, not locals
        self._ar = torch.arange(bs, device=self.param.device)
        ar = self._ar
        # Graphs of PPO objects that are unreachable but still in reference cycles stay alive
        # until the cycle collector runs; with 7 of them alive the next capture fails inside
        # hipBLASLt (tools/graph_capture_probe.py, PROBE_GC=1 clears it).  Free them first.
        gc.collect()
        s = _capture_stream(self.param.device)
        s.wait_stream(torch.cuda.current_stream(self.param.device))
        with torch.cuda.stream(s):
            for idx in warm_idx:
                self._eager_step(idx)

            def fb():
                self._forward_backward(self._perm[self._k * bs + ar])
                self._k += 1

            g1 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g1, stream=s):
                fb()
                self._apply()
            self._graphs = (g1, None)
        torch.cuda.current_stream(self.param.device).wait_stream(s)

    def _train_fused(self) -> dict:
        """All epochs and minibatches in one ``ppo_update`` launch (csrc/ppo_update.hip): the
        same randperm per epoch, losses, clipping and Adam (state kept in ``self.opt``)."""
        from . import _lib
        c = self.cfg
        obs, act, lp, adv, ret = (t.contiguous() for t in self._flat())
        n = obs.shape[0]
        bs = min(int(c.batch_size), n)
        dev = self.param.device
        perm = self._permutations(n)
        st = self.opt.state[self.param]
        if not st:  # torch's capturable-Adam state layout, created before the first step
            st["step"] = torch.zeros((), dtype=torch.float32, device=dev)
            st["exp_avg"] = torch.zeros_like(self.param, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(self.param, memory_format=torch.preserve_format)
        grp = self.opt.param_groups[0]
        hp = _lib.PPOHParams(clip_range=c.clip_range, ent_coef=c.ent_coef, vf_coef=c.vf_coef,
                             max_grad_norm=c.max_grad_norm, lr=float(grp["lr"]),
                             beta1=float(grp["betas"][0]), beta2=float(grp["betas"][1]),
                             eps=float(grp["eps"]), normalize_advantage=int(c.normalize_advantage))
        state = (self.param, st["exp_avg"], st["exp_avg_sq"], st["step"])
        snap = tuple(t.detach().clone() for t in state)  # ~120 KB: restored if the launch is lost
        steps = c.n_epochs * (-(-n // bs))
        for attempt in range(2):
            self._sums.zero_()
            _lib.check(_lib.lib().ppo_update_ws(
                _lib.ptr(self.param), _lib.ptr(st["exp_avg"]), _lib.ptr(st["exp_avg_sq"]),
                _lib.ptr(st["step"]), self.buffer.obs_dim, _lib.ptr(obs), _lib.ptr(act),
                _lib.ptr(lp), _lib.ptr(adv), _lib.ptr(ret), n, _lib.ptr(perm), c.n_epochs, bs,
                ctypes.byref(hp), _lib.ptr(self._sums), _lib.ptr(self._ws),
                _lib.current_stream(dev)), "ppo_update_ws")
            m = (self._sums / steps).tolist()
            lost = math.isnan(m[0]) and m[3] < 0
            # the ranks decide together: a retry (or the raise below) on one rank only would leave
            # the others blocked in the next collective
            if self.world > 1:
                lost = pdist.max_over_ranks(1.0 if lost else 0.0, dev) > 0
            if not lost:
                break
            # a norm exchange timed out (include/fenv.h): every rank restores and runs again
            self.exchange_retries += 1
            with torch.no_grad():
                for t, s in zip(state, snap):
                    t.copy_(s)
        bad = math.isnan(m[0])
        if self.world > 1:  # any rank's NaN makes every rank raise
            bad = pdist.max_over_ranks(1.0 if bad else 0.0, dev) > 0
        if bad:  # leave the pre-update parameters and Adam state, not NaN-poisoned ones
            with torch.no_grad():
                for t, s in zip(state, snap):
                    t.copy_(s)
            if not math.isnan(m[0]):
                raise RuntimeError("fused PPO update failed on another rank")
        if math.isnan(m[0]):
            raise RuntimeError("fused PPO update: NaN policy loss (" +
                               ("the two-CU launch's gradient-norm exchange timed out twice)"
                                if m[3] < 0 else "the update diverged)"))
        self.stats = dict(policy_gradient_loss=m[0], value_loss=m[1], entropy_loss=m[2],
                          clip_fraction=m[3])
        return self.stats

    def train(self) -> dict:
        """SB3 ``PPO.train``: n_epochs over shuffled minibatches of the rollout buffer (the same
        randperm per epoch as ``RolloutBuffer.get``) -- with several ranks, of the gathered global
        buffer, identically on every rank.  Full minibatches replay the captured graph; a
        trailing partial minibatch runs eagerly.  Losses are summed on the device and read once
        at the end."""
        if self.sharded:
            self.stats = self._dp.run(self.param, self.opt, self._flat())
            return self.stats
        self.gather_samples()
        if self.use_fused and self.cfg.batch_size <= 64:
            return self._train_fused()
        c = self.cfg
        n = self._flat()[0].shape[0]
        bs = min(int(c.batch_size), n)
        nfull, rem = divmod(n, bs)
        self._sums.zero_()
        steps = 0
        graph = self.use_graph and bs == c.batch_size and nfull > 0
        perms = self._permutations(n)
        for e in range(c.n_epochs):
            self._perm.copy_(perms[e])
            self._k.zero_()
            first = 0
            if graph and self._graphs is None:
                warm = min(3, nfull)
                self._capture([self._perm[i * bs:(i + 1) * bs] for i in range(warm)])
                first = warm
                self._k.fill_(warm)
            for i in range(first, nfull):
                if graph:
                    self._graphs[0].replay()
                else:
                    self._eager_step(self._perm[i * bs:(i + 1) * bs])
            if rem:
                self._eager_step(self._perm[nfull * bs:])
            steps += nfull + (1 if rem else 0)
        m = (self._sums / steps).tolist()
        self.stats = dict(policy_gradient_loss=m[0], value_loss=m[1], entropy_loss=m[2],
                          clip_fraction=m[3])
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
                    cb.on_steps(self, self.cfg.n_steps, self.total_envs)
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
                "n_envs": self.total_envs, "seed": self.seed}

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
        sd, data, opt_sd = ckpt.load_sb3_zip(path, with_optimizer=True)
        if cfg is None:
            cfg = PPOConfig(**ckpt.plain_hyperparameters(data, PPOConfig))
        model = cls(env, cfg, seed=seed)
        model.policy.load_state_dict(sd)
        # Adam moments and step count (SB3's per-tensor policy.optimizer.pth -> the flat state)
        flat = ckpt.optimizer_state_to_flat(model.policy.param_shapes(), opt_sd, model.param.device)
        if flat is not None:
            st = model.opt.state[model.param]
            st["step"] = flat["step"].to(torch.float32)
            st["exp_avg"] = flat["exp_avg"]
            st["exp_avg_sq"] = flat["exp_avg_sq"]
        # timestep counter: SB3 keeps num_timesteps in ``data``
        t = int(data.get("num_timesteps", 0)) if isinstance(data.get("num_timesteps", 0), int) else 0
        model.loaded_num_timesteps = t
        model.collector.num_timesteps = t // model.total_envs * env.num_envs
        return model
