"""Data-parallel PPO update: the gradient all-reduce of SURVEY §8(e)(2) / the north star ("RCCL
over xGMI used only for all-reducing policy gradients and episode statistics").

The reference trains one SB3 PPO process (/root/reference/vectorized_env.py:126-137: n_steps 10,
batch 64, 10 epochs).  With G ranks, each holding the rollout samples of its formation shard, this
update keeps the samples where they are and splits every GLOBAL minibatch of ``batch_size``
samples over the ranks, ``batch_size / G`` rows each:

  per update   one randperm of its own n_r samples per epoch on every rank; the global
               minibatches' advantage mean / std from two all-reduces of [n_epochs, M] partial
               sums (SB3 normalises advantages per minibatch, so ranks need the global values);
  per minibatch  every rank: forward + backward of its rows with the loss means taken over the
               global minibatch (``ppo_grad`` on the fused two-CU kernel, or torch autograd) ->
               ONE all-reduce (SUM) of the flat 9,669-float gradient -> clip_grad_norm_ + Adam on
               the reduced gradient (``ppo_apply``, or torch), identically on every rank, so the
               parameters and Adam state stay replicated;
  per update   one all-reduce of the four loss sums.

The result equals the single-process update whose minibatch j is the concatenation, in rank
order, of the ranks' j-th row sets -- to summation order (tests/test_distributed.py).  Uneven
shards: M = ceil(max n_r / b_local) minibatches per epoch on every rank (the same collective
count everywhere); a rank whose rows ran out contributes a zero gradient.

Cost model (docs/design_history_r1_r4.md §6): the replicated path (ppo.py) all-gathers every sample once per update
and runs all n / batch_size x n_epochs minibatches on every rank; this path moves 38.7 KB per
minibatch per rank through RCCL and divides the per-rank forward/backward work by G, at the price
of one collective per minibatch.  The minibatch sequence is SB3's and stays sequential either way.
"""
from __future__ import annotations

import ctypes
import math

import torch
import torch.distributed as dist

from . import distributed as pdist


def minibatch_plan(n_local: list[int], batch_size: int, world: int):
    """(b_local, M, rows[r][j], b_global[j]): each rank's row count in global minibatch j."""
    if batch_size % world:
        raise ValueError(f"sharded update: batch_size {batch_size} must be a multiple of the "
                         f"world size {world}")
    b = batch_size // world
    M = max(-(-n // b) for n in n_local)
    rows = [[max(0, min(b, n - j * b)) for j in range(M)] for n in n_local]
    bg = [sum(rows[r][j] for r in range(world)) for j in range(M)]
    return b, M, rows, bg


class ShardedUpdate:
    """One rank's side of the data-parallel update (see the module docstring).

    ``fused``: the gradient and the clip + Adam step on the HIP kernels (``ppo_grad`` /
    ``ppo_apply``, include/fenv.h); otherwise torch autograd + ``opt`` (any device)."""

    def __init__(self, cfg, obs_dim: int, n_local: list[int], seed: int, device,
                 fused: bool = False, gen: torch.Generator | None = None):
        self.cfg = cfg
        self.D = int(obs_dim)
        self.world, self.rank = pdist.world_rank()
        if len(n_local) != self.world:
            raise ValueError("n_local needs one sample count per rank")
        self.n_local = [int(n) for n in n_local]
        self.b, self.M, self.rows, self.bg = minibatch_plan(self.n_local, int(cfg.batch_size),
                                                            self.world)
        self.device = torch.device(device)
        # each rank shuffles its own samples: a generator per (seed, rank).  `gen` (one rank):
        # the caller's generator -- ppo.PPO passes the one its replicated path draws SB3's
        # per-epoch randperm from, so at world 1 both modes run the same minibatches
        self.gen = gen if gen is not None else torch.Generator(device=self.device).manual_seed(
            (int(seed) * 1_000_003 + self.rank) & 0x7FFFFFFFFFFFFFFF)
        self.fused = bool(fused)
        self.sums = torch.zeros(4, dtype=torch.float64, device=self.device)

    # ------------------------------------------------------------------ per update
    def permutations(self) -> torch.Tensor:
        """[n_epochs, n_local] int64: one randperm per epoch (ppo.epoch_permutations' draws)."""
        n = self.n_local[self.rank]
        perm = torch.empty((self.cfg.n_epochs, n), dtype=torch.long, device=self.device)
        for e in range(self.cfg.n_epochs):
            perm[e].copy_(torch.randperm(n, device=self.device, generator=self.gen))
        return perm

    def advantage_stats(self, adv: torch.Tensor, perm: torch.Tensor):
        """Global minibatch advantage mean and (unbiased) std, [n_epochs, M] each, from two
        all-reduces of per-rank partial sums (two-pass, as torch's std)."""
        E, M, b = self.cfg.n_epochs, self.M, self.b
        n = self.n_local[self.rank]
        pad = torch.zeros((E, M * b), dtype=torch.float64, device=self.device)
        mask = torch.zeros((E, M * b), dtype=torch.float64, device=self.device)
        pad[:, :n] = adv[perm].double()
        mask[:, :n] = 1.0
        pad, mask = pad.view(E, M, b), mask.view(E, M, b)
        bg = torch.tensor(self.bg, dtype=torch.float64, device=self.device)
        s = pad.sum(-1)
        if self.world > 1:
            dist.all_reduce(s)
        mean = s / bg
        d = ((pad - mean[..., None]) * mask).pow(2).sum(-1)
        if self.world > 1:
            dist.all_reduce(d)
        std = (d / (bg - 1).clamp(min=1)).sqrt()
        return mean.float(), std.float()

    # ------------------------------------------------------------------ one minibatch, eager
    def _local_grad_eager(self, param, samples, idx, bg: int, mean: float, std: float) -> None:
        from .ppo import evaluate_actions
        c = self.cfg
        obs, act, old_lp, adv, ret = (t[idx] for t in samples)
        ent_once = self.rank == 0
        param.grad = torch.zeros_like(param)
        if idx.numel() == 0 and not ent_once:
            return
        values, log_prob, entropy = evaluate_actions(self.D, param, obs, act)
        if c.normalize_advantage and bg > 1:
            adv = (adv - mean) / (std + 1e-8)
        ratio = torch.exp(log_prob - old_lp)
        l1 = adv * ratio
        l2 = adv * torch.clamp(ratio, 1 - c.clip_range, 1 + c.clip_range)
        policy_loss = -torch.min(l1, l2).sum() / bg
        value_loss = ((ret - values) ** 2).sum() / bg
        loss = policy_loss + c.vf_coef * value_loss
        ent = torch.zeros((), dtype=torch.float64, device=param.device)
        if ent_once:  # SB3's entropy loss is the same for every sample: one rank adds it
            log_std = param[-2:]
            entropy_loss = -(0.5 + 0.5 * math.log(2 * math.pi) + log_std).sum()
            loss = loss + c.ent_coef * entropy_loss
            ent = entropy_loss.detach().double()
        loss.backward()
        cf = (torch.abs(ratio - 1) > c.clip_range).float().sum() / bg
        self.sums += torch.stack([policy_loss.detach().double(), value_loss.detach().double(),
                                  ent, cf.double()])

    # ------------------------------------------------------------------ the update
    def run(self, param, opt, samples) -> dict:
        """One PPO update over this rank's ``samples`` = (obs [n, D], actions [n, 2],
        old_log_prob [n], advantages [n], returns [n]); ``param`` (flat, with ``opt`` its Adam)
        is updated in place, identically on every rank.  Returns the mean losses."""
        c = self.cfg
        n = self.n_local[self.rank]
        if samples[0].shape[0] != n:
            raise ValueError(f"rank {self.rank}: {samples[0].shape[0]} samples, plan says {n}")
        perm = self.permutations()
        mean, std = self.advantage_stats(samples[3], perm)
        mean_h, std_h = mean.tolist(), std.tolist()  # one device->host copy per update
        self.sums.zero_()
        grad = torch.zeros_like(param)
        fused = self.fused and self._fused_setup(param, opt)
        for e in range(c.n_epochs):
            for j in range(self.M):
                bl = self.rows[self.rank][j]
                idx = perm[e, j * self.b:j * self.b + bl]
                if fused:
                    self._local_grad_fused(param, samples, idx, bl, self.bg[j], mean_h[e][j],
                                           std_h[e][j], grad)
                else:
                    self._local_grad_eager(param, samples, idx, self.bg[j], mean_h[e][j],
                                           std_h[e][j])
                    grad = param.grad
                if self.world > 1:
                    dist.all_reduce(grad)
                if fused:
                    self._apply_fused(param, grad)
                else:
                    torch.nn.utils.clip_grad_norm_([param], c.max_grad_norm)
                    opt.step()
        if self.world > 1:
            dist.all_reduce(self.sums)
        m = (self.sums / (c.n_epochs * self.M)).tolist()
        return dict(policy_gradient_loss=m[0], value_loss=m[1], entropy_loss=m[2],
                    clip_fraction=m[3])

    # ------------------------------------------------------------------ fused kernels
    def _fused_setup(self, param, opt) -> bool:
        from . import _lib
        st = opt.state[param]
        if not st:
            st["step"] = torch.zeros((), dtype=torch.float32, device=param.device)
            st["exp_avg"] = torch.zeros_like(param, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(param, memory_format=torch.preserve_format)
        grp = opt.param_groups[0]
        c = self.cfg
        self._hp = _lib.PPOHParams(clip_range=c.clip_range, ent_coef=c.ent_coef,
                                   vf_coef=c.vf_coef, max_grad_norm=c.max_grad_norm,
                                   lr=float(grp["lr"]), beta1=float(grp["betas"][0]),
                                   beta2=float(grp["betas"][1]), eps=float(grp["eps"]),
                                   normalize_advantage=int(c.normalize_advantage))
        self._st = st
        return True

    def _local_grad_fused(self, param, samples, idx, bl, bg, mean, std, grad) -> None:
        from . import _lib
        obs, act, lp, adv, ret = samples
        _lib.check(_lib.lib().ppo_grad(
            _lib.ptr(param), self.D, _lib.ptr(obs), _lib.ptr(act), _lib.ptr(lp), _lib.ptr(adv),
            _lib.ptr(ret), _lib.ptr(idx) if bl else None, int(bl), int(bg), float(mean),
            float(std), int(self.cfg.normalize_advantage), int(self.rank == 0),
            ctypes.byref(self._hp), _lib.ptr(grad), _lib.ptr(self.sums),
            _lib.current_stream(param.device)), "ppo_grad")

    def _apply_fused(self, param, grad) -> None:
        from . import _lib
        st = self._st
        _lib.check(_lib.lib().ppo_apply(
            _lib.ptr(param), _lib.ptr(st["exp_avg"]), _lib.ptr(st["exp_avg_sq"]),
            _lib.ptr(st["step"]), _lib.ptr(grad), self.D, ctypes.byref(self._hp),
            _lib.current_stream(param.device)), "ppo_apply")
