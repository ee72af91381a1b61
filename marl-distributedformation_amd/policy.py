"""Actor-critic MLP policy (SB3 ``MlpPolicy`` for a Box action space) on the gfx950 matrix cores.

The reference trains ``PPO('MlpPolicy', env, n_steps=10, learning_rate=1e-3, ent_coef=0.01)``
(vectorized_env.py:126-131) and plays back with ``model.predict(obs, deterministic=True)``
(visualize_policy.py:16).  :class:`MlpPolicy` keeps SB3's parameter names (``state_dict`` /
``load_state_dict`` interoperate with an SB3 ``policy.pth``) and runs the forward pass --
both networks, Gaussian sampling, log-prob and action clipping -- in one HIP kernel
(``policy_forward`` in include/fenv.h).  Parameters live in one flat fp32 device buffer.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import _lib

HID = 64

# SB3 state_dict names and shapes, in the flat-buffer order of include/fenv.h
PARAM_SPECS = [
    ("mlp_extractor.policy_net.0.weight", (HID, "D")),
    ("mlp_extractor.policy_net.0.bias", (HID,)),
    ("mlp_extractor.policy_net.2.weight", (HID, HID)),
    ("mlp_extractor.policy_net.2.bias", (HID,)),
    ("mlp_extractor.value_net.0.weight", (HID, "D")),
    ("mlp_extractor.value_net.0.bias", (HID,)),
    ("mlp_extractor.value_net.2.weight", (HID, HID)),
    ("mlp_extractor.value_net.2.bias", (HID,)),
    ("action_net.weight", (2, HID)),
    ("action_net.bias", (2,)),
    ("value_net.weight", (1, HID)),
    ("value_net.bias", (1,)),
    ("log_std", (2,)),
]


def _shape(shp, D):
    return tuple(D if s == "D" else s for s in shp)


def param_shapes(obs_dim: int):
    """[(SB3 name, shape)] in flat-buffer order for observation size ``obs_dim`` (no device)."""
    return [(k, _shape(shp, obs_dim)) for k, shp in PARAM_SPECS]


class MlpPolicy:
    """Flat-parameter actor-critic with SB3 naming; forward on the HIP kernel."""

    def __init__(self, obs_dim: int = 8, device=None, seed: int = 0, log_std_init: float = 0.0):
        if obs_dim not in (6, 8):
            raise ValueError("obs_dim must be 6 or 8 (vectorized_env.py:28-31)")
        self.obs_dim = obs_dim
        self.device = _lib.require_device(device)
        n = int(_lib.lib().policy_param_count(obs_dim))
        self.flat = torch.zeros(n, dtype=torch.float32, device=self.device)
        self._views = {}
        o = 0
        for k, shp in PARAM_SPECS:
            s = _shape(shp, obs_dim)
            m = int(np.prod(s))
            self._views[k] = self.flat[o:o + m].view(s)
            o += m
        assert o == n
        self.reset_parameters(seed, log_std_init)
        self._offset = 0
        self._host = {}  # predict(): device-mapped host arrays per batch size (_lib.HostBlock)
        self.sample_seed = int(seed)

    # ---------------------------------------------------------------- parameters
    def param_shapes(self):
        """[(SB3 name, shape)] in flat-buffer order."""
        return [(k, _shape(shp, self.obs_dim)) for k, shp in PARAM_SPECS]

    def reset_parameters(self, seed: int = 0, log_std_init: float = 0.0) -> None:
        """SB3's init: orthogonal weights (gain sqrt(2) hidden, 0.01 action head, 1 value head),
        zero biases, log_std = log_std_init (SB3 default 0.0; note vectorized_env.py:133 sets
        log_std_init after construction, which SB3 ignores)."""
        g = torch.Generator().manual_seed(seed)
        for k, v in self._views.items():
            if k.endswith("weight"):
                gain = (0.01 if k.startswith("action_net")
                        else 1.0 if k.startswith("value_net") else math.sqrt(2))
                w = torch.empty(tuple(v.shape))
                torch.nn.init.orthogonal_(w, gain=gain, generator=g)
                v.copy_(w)
            elif k == "log_std":
                v.fill_(log_std_init)
            else:
                v.zero_()

    def state_dict(self) -> dict:
        return {k: v.detach().clone().cpu() for k, v in self._views.items()}

    def load_state_dict(self, sd: dict, strict: bool = True) -> None:
        """Accepts an SB3 policy state_dict (extra keys such as features extractors ignored)."""
        for k, v in self._views.items():
            if k not in sd:
                if strict:
                    raise KeyError(f"missing parameter {k}")
                continue
            t = torch.as_tensor(sd[k], dtype=torch.float32)
            if tuple(t.shape) != tuple(v.shape):
                raise ValueError(f"{k}: shape {tuple(t.shape)} != {tuple(v.shape)}")
            v.copy_(t)

    @classmethod
    def from_checkpoint(cls, path: str, device=None) -> "MlpPolicy":
        """Policy from an SB3 model zip (``rl_model_*_steps.zip``, ours or SB3's; only its
        ``policy.pth`` is read, with torch.load(weights_only=True)): visualize_policy.py:35."""
        from .checkpoint import load_sb3_zip
        sd, _ = load_sb3_zip(path)
        D = int(sd["mlp_extractor.policy_net.0.weight"].shape[1])
        pol = cls(D, device=device)
        pol.load_state_dict(sd)
        return pol

    def parameters_flat(self) -> torch.Tensor:
        return self.flat

    # ---------------------------------------------------------------- forward
    def forward(self, obs: torch.Tensor, deterministic: bool = False, out: dict | None = None,
                seed: int | None = None, offset: int | None = None, row0: int = 0) -> dict:
        """obs [B, D] float32 on the device -> dict(mu, value, action, log_prob, clipped).

        ``action`` is the unclipped sample (what SB3 stores in the rollout buffer); ``clipped``
        is what collect_rollouts passes to env.step.  Each call advances the noise offset.
        Row r's noise is keyed by the global row ``row0 + r`` (a shard passes its first agent)."""
        if obs.dim() != 2 or obs.shape[1] != self.obs_dim:
            raise ValueError(f"obs must be [B, {self.obs_dim}]")
        if obs.dtype != torch.float32 or obs.device != self.device:
            raise TypeError(f"obs must be float32 on {self.device}")
        obs = obs.contiguous()
        B = obs.shape[0]
        dev = self.device
        if out is not None:
            for k, shp in (("mu", (B, 2)), ("value", (B,)), ("action", (B, 2)),
                           ("log_prob", (B,)), ("clipped", (B, 2))):
                t = out.get(k)
                if t is not None and (t.device != dev or t.dtype != torch.float32
                                      or tuple(t.shape) != shp or not t.is_contiguous()):
                    raise ValueError(f"out[{k!r}] must be a contiguous float32 {shp} tensor on {dev}")
        if out is None:
            out = dict(mu=torch.empty((B, 2), device=dev), value=torch.empty(B, device=dev),
                       action=torch.empty((B, 2), device=dev), log_prob=torch.empty(B, device=dev),
                       clipped=torch.empty((B, 2), device=dev))
        if offset is None:
            offset = self._offset
            self._offset += 1
        if B == 0:  # nothing to launch (an empty tensor's data pointer is NULL)
            return out
        s = self.sample_seed if seed is None else seed
        _lib.check(_lib.lib().policy_forward(
            _lib.ptr(self.flat), self.obs_dim, _lib.ptr(obs), B, int(row0), _lib.ptr(out.get("mu")),
            _lib.ptr(out.get("value")), _lib.ptr(out.get("action")), _lib.ptr(out.get("log_prob")),
            _lib.ptr(out.get("clipped")), int(s) & 0xFFFFFFFFFFFFFFFF, int(offset),
            int(bool(deterministic)), _lib.current_stream(dev)), "policy_forward")
        return out

    __call__ = forward

    def predict(self, observation, deterministic: bool = True):
        """SB3 ``predict``: numpy obs [B, D] -> (clipped actions numpy [B, 2], None).

        The kernel reads the observations and writes the actions in device-mapped host memory
        (``_lib.HostBlock``): observations a FormationEnv's numpy face returned are read in place,
        others are first copied into the policy's block; the actions come back as a new array.
        Same bits and the same noise offset advance as ``forward(...)["clipped"]`` (an empty batch
        included: it advances the offset and launches nothing)."""
        if isinstance(observation, torch.Tensor) and observation.is_cuda:
            return self.forward(observation, deterministic=deterministic)["clipped"].cpu().numpy(), None
        obs = np.asarray(observation, np.float32)
        if obs.ndim != 2 or obs.shape[1] != self.obs_dim:
            raise ValueError(f"obs must be [B, {self.obs_dim}]")
        B = obs.shape[0]
        if B == 0:
            self._offset += 1  # as forward() on an empty batch
            return np.zeros((0, 2), np.float32), None
        host = self._host.get(B)
        if host is None:
            host = _lib.HostBlock(self.device, [("obs", np.float32, (B, self.obs_dim)),
                                                ("clipped", np.float32, (B, 2))])
            self._host = {B: host}  # one batch size cached (playback and SB3 loops keep theirs)
        d_obs = _lib.device_address(obs, self.device)
        if d_obs is None:
            np.copyto(host.obs, obs)
            d_obs = host.dev("obs")
        offset = self._offset
        self._offset += 1
        dev = self.device
        _lib.check(_lib.lib().policy_forward(
            _lib.ptr(self.flat), self.obs_dim, d_obs, B, 0, None, None, None, None,
            host.dev("clipped"), int(self.sample_seed) & 0xFFFFFFFFFFFFFFFF, int(offset),
            int(bool(deterministic)), _lib.current_stream(dev)), "policy_forward")
        torch.cuda.current_stream(dev).synchronize()
        return host.clipped.copy(), None

