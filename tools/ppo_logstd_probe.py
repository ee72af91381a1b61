"""where does the fused PPO update's log_std path leave torch?

Along the reference-config trajectory (1,000 x 5 agents, n_steps 10, batch 64, 10 epochs = 7,820
minibatches; the seeds of tests/test_gpu_ppo_dp.py::test_fused_update_vs_torch_at_reference_config)
the torch fp32 update is stepped, and at EVERY minibatch, from torch's own parameters:
  * g64 = float64 autograd of the SB3 loss (the truth),
  * g32 = torch fp32 autograd (what the test's torch leg computes),
  * gk  = the fused kernel's gradient of the same minibatch (ppo_grad: the kernel's forward, loss
          and backward in gradient mode, same rows, advantages normalised like torch),
and the kernel's clip + Adam step (ppo_apply) is compared with torch's clip + Adam from the same
state and gradient.  Per parameter group it reports the signed error of gk and g32 against g64
(mean and rms over the trajectory, in units of |g64|), so a systematic (biased) error shows as a
mean far above rms / sqrt(K), and the Adam step's max relative difference.

    python tools/ppo_logstd_probe.py [minibatches]      -> JSON summary on stdout
"""
import ctypes
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pkgload  # noqa: E402

pkg = pkgload.load()
from importlib import import_module  # noqa: E402

ve = import_module(pkg.__name__ + ".vectorized_env")
ppo_mod = import_module(pkg.__name__ + ".ppo")
L = import_module(pkg.__name__ + "._lib")
DEV = "cuda:0"
K = int(sys.argv[1]) if len(sys.argv) > 1 else 7820

env = ve.FormationEnv({"num_formation": 1000, "num_agents_per_formation": 5, "goal_in_obs": True},
                      device=DEV, seed=2, reset_mode="philox")
m = ppo_mod.PPO(env, ppo_mod.PPOConfig(), seed=3, use_graph=False, use_fused=False)
c = m.cfg
with torch.no_grad():
    m.collector.collect()
obs, act, old_lp, adv, ret = (t.contiguous() for t in m._flat())
n = obs.shape[0]
perm = ppo_mod.epoch_permutations(n, c.n_epochs, torch.Generator(device=DEV).manual_seed(3), DEV)
D = obs.shape[1]
P = m.param.numel()
hp = L.PPOHParams(clip_range=c.clip_range, ent_coef=c.ent_coef, vf_coef=c.vf_coef,
                  max_grad_norm=c.max_grad_norm, lr=c.learning_rate, beta1=0.9, beta2=0.999,
                  eps=1e-5, normalize_advantage=1)
lib = L.lib()
stream = L.current_stream(torch.device(DEV))

# parameter groups (policy.param_shapes order)
groups, o = [], 0
for k, shp in m.policy.param_shapes():
    nn_ = math.prod(shp)
    groups.append((k.split(".")[-2] + "." + k.split(".")[-1] if "." in k else k, o, o + nn_))
    o += nn_


def loss_grad(flat, idx, dtype):
    p = flat.detach().to(dtype).clone().requires_grad_(True)
    o_, a_, lp_, ad_, r_ = (t[idx].to(dtype) for t in (obs, act, old_lp, adv, ret))
    values, log_prob, entropy = ppo_mod.evaluate_actions(m.policy, p, o_, a_)
    ad_ = (ad_ - ad_.mean()) / (ad_.std() + 1e-8)
    ratio = torch.exp(log_prob - lp_)
    l1, l2 = ad_ * ratio, ad_ * torch.clamp(ratio, 1 - c.clip_range, 1 + c.clip_range)
    loss = (-torch.min(l1, l2).mean() + c.ent_coef * -torch.mean(entropy)
            + c.vf_coef * torch.nn.functional.mse_loss(r_, values))
    loss.backward()
    return p.grad.detach()


param = m.param
opt = torch.optim.Adam([param], lr=c.learning_rate, eps=1e-5, capturable=True)
gk = torch.zeros(P, dtype=torch.float32, device=DEV)
stats = torch.zeros(4, dtype=torch.float64, device=DEV)
G = len(groups)
acc = {w: {"sum": torch.zeros(G, dtype=torch.float64, device=DEV),
           "sq": torch.zeros(G, dtype=torch.float64, device=DEV)} for w in ("k", "t32")}
ls_err = []  # per-minibatch log_std signed errors (kernel, torch32), in units of |g64_logstd|
adam_rel = 0.0
first_bad = None
kmb = 0
for e in range(c.n_epochs):
    for s0 in range(0, n, c.batch_size):
        if kmb >= K:
            break
        idx = perm[e, s0:s0 + c.batch_size].contiguous()
        B = idx.numel()
        g64 = loss_grad(param, idx, torch.float64)
        g32 = loss_grad(param, idx, torch.float32).double()
        a = adv[idx]
        mean, std = float(a.mean()), float(a.std())
        L.check(lib.ppo_grad(L.ptr(param), D, L.ptr(obs), L.ptr(act), L.ptr(old_lp), L.ptr(adv),
                             L.ptr(ret), L.ptr(idx), B, B, mean, std, 1, 1, ctypes.byref(hp),
                             L.ptr(gk), L.ptr(stats), stream), "ppo_grad")
        gkd = gk.double()
        for w, gg in (("k", gkd), ("t32", g32)):
            for gi, (_, lo, hi) in enumerate(groups):
                d = gg[lo:hi] - g64[lo:hi]
                scale = g64[lo:hi].abs().max().clamp(min=1e-30)
                acc[w]["sum"][gi] += (d.sum() / (scale * (hi - lo)))
                acc[w]["sq"][gi] += (d.pow(2).mean() / scale ** 2)
        sc = g64[-2:].abs().clamp(min=1e-30)
        ek = ((gkd[-2:] - g64[-2:]) / sc).tolist()
        et = ((g32[-2:] - g64[-2:]) / sc).tolist()
        ls_err.append((ek, et))
        if first_bad is None and max(abs(x) for x in ek) > 10 * max(1e-6, max(abs(x) for x in et)):
            first_bad = {"minibatch": kmb, "kernel_rel": ek, "torch32_rel": et,
                         "g64_logstd": g64[-2:].tolist()}
        # the kernel's clip + Adam from torch's state and torch's fp32 gradient
        st = opt.state[param]
        if st:
            pk, mk, vk, sk = (param.detach().clone(), st["exp_avg"].clone(),
                              st["exp_avg_sq"].clone(), st["step"].clone())
        else:
            pk, mk, vk = param.detach().clone(), torch.zeros_like(param), torch.zeros_like(param)
            sk = torch.zeros((), dtype=torch.float32, device=DEV)
        g32f = g32.float().contiguous()
        L.check(lib.ppo_apply(L.ptr(pk), L.ptr(mk), L.ptr(vk), L.ptr(sk), L.ptr(g32f), D,
                              ctypes.byref(hp), stream), "ppo_apply")
        param.grad = g32f.clone()
        torch.nn.utils.clip_grad_norm_([param], c.max_grad_norm)
        opt.step()
        # |kernel step - torch step| over lr (both steps are at most ~lr per element)
        adam_rel = max(adam_rel, (param.detach() - pk).abs().max().item() / c.learning_rate)
        kmb += 1
torch.cuda.synchronize()
Kd = float(kmb)
out = {"minibatches": kmb, "groups": {}}
for gi, (name, lo, hi) in enumerate(groups):
    out["groups"][name] = {
        w: {"mean_signed_err": acc[w]["sum"][gi].item() / Kd,
            "rms_err": math.sqrt(acc[w]["sq"][gi].item() / Kd)} for w in ("k", "t32")}
ek = torch.tensor([x[0] for x in ls_err], dtype=torch.float64)
et = torch.tensor([x[1] for x in ls_err], dtype=torch.float64)
out["log_std"] = {"kernel": {"mean": ek.mean(0).tolist(), "rms": ek.pow(2).mean(0).sqrt().tolist(),
                             "max": ek.abs().max(0).values.tolist()},
                  "torch32": {"mean": et.mean(0).tolist(), "rms": et.pow(2).mean(0).sqrt().tolist(),
                              "max": et.abs().max(0).values.tolist()}}
out["first_minibatch_kernel_10x_torch32"] = first_bad
out["adam_max_abs_diff_over_lr"] = adam_rel
print(json.dumps(out, indent=1))
