"""VERDICT r3 next #3, second probe: is the fused PPO update's whole step (gradient, clip, Adam)
biased against torch's?  Along the reference-config trajectory (the seeds of
tests/test_gpu_ppo_dp.py::test_fused_update_vs_torch_at_reference_config), from torch's own state
at EVERY minibatch, three one-step updates are compared:
  * d64 -- float64: autograd of the SB3 loss, clip_grad_norm_, Adam with torch's formulas and the
           Python-float betas (the truth);
  * d32 -- torch fp32: the trajectory's own step (autograd + clip_grad_norm_ + capturable Adam);
  * dk  -- the fused kernel: ppo_update_ws over just this minibatch's rows (one epoch, identity
           permutation) from copies of torch's parameters and Adam state.
Per parameter group: the mean over the trajectory of the signed relative step error
(d - d64) * sign(d64) / |d64| over the elements with |d64| > 1e-3 lr ("overshoot": > 0 means
steps systematically too long) and its rms.  A coherent error -- one that is the same sign at every
step -- shows as |mean| >> rms / sqrt(elements).

    python tools/ppo_step_probe.py [minibatches]      -> JSON summary on stdout
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
n, D = obs.shape
perm = ppo_mod.epoch_permutations(n, c.n_epochs, torch.Generator(device=DEV).manual_seed(3), DEV)
P = m.param.numel()
B1, B2, EPS, LR = 0.9, 0.999, 1e-5, c.learning_rate
hp = L.PPOHParams(clip_range=c.clip_range, ent_coef=c.ent_coef, vf_coef=c.vf_coef,
                  max_grad_norm=c.max_grad_norm, lr=LR, beta1=B1, beta2=B2, eps=EPS,
                  normalize_advantage=1)
lib = L.lib()
stream = L.current_stream(torch.device(DEV))
ws = torch.zeros(int(lib.ppo_workspace_bytes()), dtype=torch.uint8, device=DEV)
groups, o = [], 0
for k, shp in m.policy.param_shapes():
    nn_ = math.prod(shp)
    groups.append((k, o, o + nn_))
    o += nn_


def grad(flat, idx, dtype):
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
opt = torch.optim.Adam([param], lr=LR, eps=EPS, capturable=True)
G = len(groups)
acc = {w: {"sum": torch.zeros(G, dtype=torch.float64, device=DEV),
           "sq": torch.zeros(G, dtype=torch.float64, device=DEV),
           "cnt": torch.zeros(G, dtype=torch.float64, device=DEV)} for w in ("k", "t32")}
stats = torch.zeros(4, dtype=torch.float64, device=DEV)
kmb = 0
for e in range(c.n_epochs):
    for s0 in range(0, n, c.batch_size):
        if kmb >= K:
            break
        idx = perm[e, s0:s0 + c.batch_size].contiguous()
        B = idx.numel()
        st = opt.state[param]
        if st:
            mk, vk, sk = st["exp_avg"].clone(), st["exp_avg_sq"].clone(), st["step"].clone()
        else:
            mk, vk = torch.zeros_like(param), torch.zeros_like(param)
            sk = torch.zeros((), dtype=torch.float32, device=DEV)
        p0 = param.detach().clone()
        # float64 step from torch's state
        g64 = grad(param, idx, torch.float64)
        nrm = g64.norm()
        g64 = g64 * min(1.0, c.max_grad_norm / (nrm.item() + 1e-6))
        t = kmb + 1
        ms, vs = mk.double(), vk.double()  # torch's state before the step
        m64_n = ms + (1 - B1) * (g64 - ms)
        v64_n = vs * B2 + (1 - B2) * g64 * g64
        d64 = -(LR / (1 - B1 ** t)) * m64_n / (v64_n.sqrt() / math.sqrt(1 - B2 ** t) + EPS)
        # the fused kernel, one minibatch from torch's state
        rows = [x[idx].contiguous() for x in (obs, act, old_lp, adv, ret)]
        pk = p0.clone()
        ar = torch.arange(B, device=DEV, dtype=torch.long)
        L.check(lib.ppo_update_ws(L.ptr(pk), L.ptr(mk), L.ptr(vk), L.ptr(sk), D,
                                  *(L.ptr(x) for x in rows), B, L.ptr(ar), 1, B,
                                  ctypes.byref(hp), L.ptr(stats), L.ptr(ws), stream),
                "ppo_update_ws")
        dk = (pk - p0).double()
        # torch's own fp32 step (the trajectory)
        param.grad = grad(param, idx, torch.float32)
        torch.nn.utils.clip_grad_norm_([param], c.max_grad_norm)
        opt.step()
        d32 = (param.detach() - p0).double()
        sel = d64.abs() > 1e-3 * LR
        sg = torch.sign(d64)
        for w, d in (("k", dk), ("t32", d32)):
            r = torch.where(sel, (d - d64) * sg / d64.abs().clamp(min=1e-30), torch.zeros_like(d))
            for gi, (_, lo, hi) in enumerate(groups):
                acc[w]["sum"][gi] += r[lo:hi].sum()
                acc[w]["sq"][gi] += r[lo:hi].pow(2).sum()
                acc[w]["cnt"][gi] += sel[lo:hi].sum()
        kmb += 1
torch.cuda.synchronize()
out = {"minibatches": kmb, "definition": "signed relative step error vs float64, mean over "
       "elements with |d64| > 1e-3 lr; > 0 = steps too long", "groups": {}}
tot = {w: [0.0, 0.0, 0.0] for w in ("k", "t32")}
for gi, (name, lo, hi) in enumerate(groups):
    row = {}
    for w in ("k", "t32"):
        cnt = max(1.0, acc[w]["cnt"][gi].item())
        s, q = acc[w]["sum"][gi].item(), acc[w]["sq"][gi].item()
        row[w] = {"mean": s / cnt, "rms": math.sqrt(q / cnt), "n": int(cnt)}
        tot[w][0] += s
        tot[w][1] += q
        tot[w][2] += cnt
    out["groups"][name] = row
out["all"] = {w: {"mean": tot[w][0] / tot[w][2], "rms": math.sqrt(tot[w][1] / tot[w][2]),
                  "n": int(tot[w][2])} for w in ("k", "t32")}
print(json.dumps(out, indent=1))
