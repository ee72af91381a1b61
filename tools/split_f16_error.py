"""Numerical justification of the split-f16 policy MFMA (csrc/policy_device.h), on the CPU.

Emulates what the kernel computes.  The hidden layers carry r = 1/(1 + e^{2x}) instead of
tanh(x) = 1 - 2r (the next layer and the heads absorb the affine map: weights -2W, bias
b + rowsum W), and every fp32 product w*x of the two hidden layers is split:
    weights      w*2/ln2 -> hi = nearest 11-significant-bit value (ties away), lo = rtz_f16(w - hi)
    activations  x       -> hi = x truncated to 11 significant bits,      lo = rtz_f16(x - hi)
    product      hi_w*hi_x + hi_w*lo_x + lo_w*hi_x   (each exact, accumulated in fp32 -- here f64)
and compares mu / value against the fp32 torch oracle (oracle/policy_oracle.py) in units of the
GPU test tolerance |err| <= 2e-5 + 2e-5|ref| (tests/test_gpu_policy.py), over SB3-initialised
policies with perturbed weights and observation scales 1e-4 .. 40 (the test's cases).
Also reports what an f16 subnormal flush would do (it would fail; tools/mfma_f16_probe.hip shows
the hardware honours subnormals).

    python tools/split_f16_error.py
"""
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import policy_oracle as po  # noqa: E402

K = np.float32(2 / math.log(2))


def rtz16(x):
    """float32 -> float16 rounding toward zero (v_cvt_pkrtz_f16_f32)."""
    h = x.astype(np.float16)
    over = np.abs(h.astype(np.float32)) > np.abs(x)
    hb = h.view(np.uint16).copy()
    hb[over & (h != 0)] -= 1
    return hb.view(np.float16)


def hi11(x, nearest):
    u = x.astype(np.float32).view(np.uint32)
    if nearest:
        u = u + np.uint32(0x1000)
    return (u & np.uint32(0xFFFFE000)).view(np.float32)


def split(x, nearest, ftz=False):
    x = x.astype(np.float32)
    hi = rtz16(hi11(x, nearest)).astype(np.float64)
    lo = rtz16((x - hi11(x, nearest)).astype(np.float32)).astype(np.float64)
    if ftz:
        hi, lo = (np.where(np.abs(v) < 2.0 ** -14, 0.0, v) for v in (hi, lo))
    return hi, lo


def lin(W, b, x, ftz):
    Wk = (W * K).astype(np.float32)
    bk = (b * K).astype(np.float32)
    wh, wl = split(Wk, True, ftz)
    xh, xl = split(x, False, ftz)
    return (xh @ wh.T + xl @ wh.T + xh @ wl.T + bk).astype(np.float32)


def rsig(y):
    """r = 1 / (1 + 2^y), so tanh(x) = 1 - 2 r for y = x * 2/ln2 (v_exp_f32, v_add, v_rcp_f32)."""
    with np.errstate(over="ignore"):
        e = np.exp2(y.astype(np.float64)).astype(np.float32)
    return (np.float32(1) / (np.float32(1) + e)).astype(np.float32)


def lin_r(W, b, r, ftz):
    """Layer fed with r instead of tanh = 1 - 2r: W.(1 - 2r) + b = (b + rowsum W) - 2 W.r."""
    Wk = (W * K).astype(np.float32)
    bk = (b * K).astype(np.float32) + Wk.sum(axis=1, dtype=np.float32)
    W2 = (np.float32(-2) * Wk).astype(np.float32)
    wh, wl = split(W2, True, ftz)
    xh, xl = split(r, False, ftz)
    return (xh @ wh.T + xl @ wh.T + xh @ wl.T + bk).astype(np.float32)


def head_r(W, b, r):
    bb = (b + W.sum(axis=1, dtype=np.float32)).astype(np.float32)
    return (r.astype(np.float64) @ (np.float32(-2) * W).T.astype(np.float64) + bb).astype(np.float32)


def forward(sd, obs, ftz=False):
    g = {k: v.numpy() for k, v in sd.items()}
    h = rsig(lin(g["mlp_extractor.policy_net.0.weight"], g["mlp_extractor.policy_net.0.bias"], obs, ftz))
    h = rsig(lin_r(g["mlp_extractor.policy_net.2.weight"], g["mlp_extractor.policy_net.2.bias"], h, ftz))
    v = rsig(lin(g["mlp_extractor.value_net.0.weight"], g["mlp_extractor.value_net.0.bias"], obs, ftz))
    v = rsig(lin_r(g["mlp_extractor.value_net.2.weight"], g["mlp_extractor.value_net.2.bias"], v, ftz))
    mu = head_r(g["action_net.weight"], g["action_net.bias"], h)
    val = head_r(g["value_net.weight"], g["value_net.bias"], v)
    return mu, val[:, 0]


def make_policy(D, seed):
    g = torch.Generator().manual_seed(seed)
    sd = {}
    for k, shp in po.SB3_KEYS:
        shp = tuple(D if s == "D" else s for s in shp)
        if k.endswith("weight"):
            gain = (0.01 if k.startswith("action_net")
                    else 1.0 if k.startswith("value_net") else math.sqrt(2))
            w = torch.empty(shp)
            torch.nn.init.orthogonal_(w, gain=gain, generator=g)
            sd[k] = w + torch.randn(shp, generator=g) * 0.05
        elif k == "log_std":
            sd[k] = torch.randn(shp, generator=g) * 0.5
        else:
            sd[k] = torch.randn(shp, generator=g) * 0.3
    return sd


def worst(ftz):
    w = 0.0
    for seed in range(4):
        for D in (8, 6):
            for scale in (1e-4, 0.05, 1.2, 3.0, 40.0):
                sd = make_policy(D, seed)
                obs = (torch.rand((20000, D), generator=torch.Generator().manual_seed(seed)) * 2 - 1) * scale
                mu, val = po.forward(sd, obs)
                m2, v2 = forward(sd, obs.numpy(), ftz)
                for ref, got in ((mu.numpy(), m2), (val.numpy(), v2)):
                    w = max(w, float((np.abs(got - ref) / (2e-5 + 2e-5 * np.abs(ref))).max()))
    return w


if __name__ == "__main__":
    print(f"split-f16 (kernel scheme): worst |err| / tolerance = {worst(False):.3f}")
    print(f"same with f16 subnormals flushed: worst |err| / tolerance = {worst(True):.1f}")
