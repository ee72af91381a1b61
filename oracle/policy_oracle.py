"""CPU oracle for the policy forward -- TEST INFRASTRUCTURE ONLY (see oracle.py header).

Restates, with torch CPU fp32 ops, what stable-baselines3's ``ActorCriticPolicy`` computes for
``PPO('MlpPolicy', env)`` (reference call site vectorized_env.py:126; playback
visualize_policy.py:16): FlattenExtractor -> MlpExtractor (pi: Linear(D,64) Tanh Linear(64,64)
Tanh; vf: same) -> action_net Linear(64,2), value_net Linear(64,1); DiagGaussian with
state-independent log_std; ``collect_rollouts`` clips the sampled action to the Box [-1, 1].

Parity status: SB3 is not installed in this image and the reference ships no policy tests or
checkpoints, so this restatement is "parity unpinned" against SB3 itself; it
is pinned to the SB3 2.x source semantics named above.  The kernel's sampling noise comes from
its own Philox stream; :func:`philox_normals` regenerates it here.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as Fn

HID = 64

SB3_KEYS = [
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


def unflatten(flat: torch.Tensor, D: int) -> dict:
    out, o = {}, 0
    for k, shp in SB3_KEYS:
        shp = tuple(D if s == "D" else s for s in shp)
        n = int(np.prod(shp))
        out[k] = flat[o:o + n].reshape(shp)
        o += n
    assert o == flat.numel()
    return out


def forward(sd: dict, obs: torch.Tensor):
    """(mu [B,2], value [B]) in fp32 on CPU, SB3 op for op."""
    obs = obs.float()
    h = torch.tanh(Fn.linear(obs, sd["mlp_extractor.policy_net.0.weight"],
                             sd["mlp_extractor.policy_net.0.bias"]))
    h = torch.tanh(Fn.linear(h, sd["mlp_extractor.policy_net.2.weight"],
                             sd["mlp_extractor.policy_net.2.bias"]))
    v = torch.tanh(Fn.linear(obs, sd["mlp_extractor.value_net.0.weight"],
                             sd["mlp_extractor.value_net.0.bias"]))
    v = torch.tanh(Fn.linear(v, sd["mlp_extractor.value_net.2.weight"],
                             sd["mlp_extractor.value_net.2.bias"]))
    mu = Fn.linear(h, sd["action_net.weight"], sd["action_net.bias"])
    value = Fn.linear(v, sd["value_net.weight"], sd["value_net.bias"]).squeeze(-1)
    return mu, value


def log_prob(sd: dict, mu: torch.Tensor, actions: torch.Tensor) -> torch.Tensor:
    std = torch.ones_like(mu) * sd["log_std"].exp()
    dist = torch.distributions.Normal(mu, std)
    return dist.log_prob(actions).sum(dim=-1)


def _philox(ctr: np.ndarray, key: tuple[int, int]) -> np.ndarray:
    """Philox4x32-10 over uint64 arrays holding uint32 words, ctr [n,4]."""
    M = np.uint64(0xFFFFFFFF)
    c = ctr.astype(np.uint64)
    k0, k1 = np.uint64(key[0]), np.uint64(key[1])
    for _ in range(10):
        p0 = np.uint64(0xD2511F53) * c[:, 0]
        p1 = np.uint64(0xCD9E8D57) * c[:, 2]
        hi0, lo0 = p0 >> np.uint64(32), p0 & M
        hi1, lo1 = p1 >> np.uint64(32), p1 & M
        c = np.stack([hi1 ^ c[:, 1] ^ k0, lo1, hi0 ^ c[:, 3] ^ k1, lo0], axis=1)
        k0 = (k0 + np.uint64(0x9E3779B9)) & M
        k1 = (k1 + np.uint64(0xBB67AE85)) & M
    return c


def philox_normals(B: int, seed: int, offset: int, row0: int = 0) -> np.ndarray:
    """The kernel's N(0,1) noise [B, 2] (Box-Muller of Philox4x32-10 words) for global rows
    row0 .. row0+B-1, in float64."""
    rows = np.arange(row0, row0 + B, dtype=np.uint64)
    ctr = np.stack([rows & np.uint64(0xFFFFFFFF), rows >> np.uint64(32),
                    np.full(B, offset & 0xFFFFFFFF, np.uint64),
                    np.full(B, (offset >> 32) & 0xFFFFFFFF, np.uint64)], axis=1)
    r = _philox(ctr, (seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF))
    u1 = ((r[:, 0] >> np.uint64(8)) + np.uint64(1)).astype(np.float64) * 2.0 ** -24
    u2 = (r[:, 1] >> np.uint64(8)).astype(np.float64) * 2.0 ** -24
    rad = np.sqrt(-2.0 * np.log(u1))
    return np.stack([rad * np.cos(2 * math.pi * u2), rad * np.sin(2 * math.pi * u2)], axis=1)
