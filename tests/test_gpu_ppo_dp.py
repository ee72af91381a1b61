"""Round-3 PPO update tests on the GPU: per-instance exchange words (two updates on two streams of
one device), the data-parallel gradient / apply kernels (ppo_grad, ppo_apply) against torch
autograd and torch's Adam, the sharded update on the fused kernels against its eager form, and
the fused update against torch at the reference's training configuration."""
import ctypes
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def mods(pkg):
    from importlib import import_module
    return {m: import_module(pkg.__name__ + "." + m)
            for m in ("vectorized_env", "policy", "ppo", "rollout", "dp_update", "_lib")}


def _samples(n, D, seed):
    g = torch.Generator().manual_seed(seed)
    obs = (torch.rand((n, D), generator=g) * 2 - 1).to(DEV)
    act = (torch.randn((n, 2), generator=g) * 0.7).to(DEV)
    lp = (-torch.rand(n, generator=g) * 3 - 1).to(DEV)
    adv = (torch.randn(n, generator=g) * 2).to(DEV)
    ret = torch.randn(n, generator=g).to(DEV)
    return obs, act, lp, adv, ret


def _params(mods, D, seed=0):
    pol = mods["policy"].MlpPolicy(D, device=DEV, seed=seed)
    with torch.no_grad():
        pol.flat.add_(torch.randn(pol.flat.shape, generator=torch.Generator().manual_seed(seed))
                      .to(DEV) * 0.05)
        pol.flat[-2:] = torch.tensor([-0.4, 0.2], device=DEV)
    return pol.flat.clone()


def _groups(D):
    """Flat-parameter ranges of SB3's MlpPolicy tensors (csrc/policy_device.h PLayout)."""
    h = 64
    sizes = [("pi0", h * D + h), ("pi2", h * h + h), ("vf0", h * D + h), ("vf2", h * h + h),
             ("actW", 2 * h), ("actb", 2), ("valW", h), ("valb", 1), ("log_std", 2)]
    out, o = {}, 0
    for name, n in sizes:
        out[name] = (o, o + n)
        o += n
    return out


def _hp(L, cfg, lr=1e-3):
    return L.PPOHParams(clip_range=cfg.clip_range, ent_coef=cfg.ent_coef, vf_coef=cfg.vf_coef,
                        max_grad_norm=cfg.max_grad_norm, lr=lr, beta1=0.9, beta2=0.999, eps=1e-5,
                        normalize_advantage=1)


def test_two_updates_on_two_streams_equal_serial(mods):
    """Two fused updates (different parameters, samples, permutations) running concurrently on
    two streams of one device, each with its own workspace (ppo_update_ws), give the same bits as
    the same two updates run one after the other; so does the legacy ppo_update, whose exchange
    words are a stream-ordered allocation per launch (round 2 shared one set per device)."""
    L = mods["_lib"]
    lib = L.lib()
    cfg = mods["ppo"].PPOConfig()
    D, n, E = 8, 5000, 2
    jobs = []
    for k in range(2):
        smp = _samples(n, D, 10 + k)
        perm = torch.stack([torch.randperm(n, generator=torch.Generator().manual_seed(20 + 2 * k + e))
                            for e in range(E)]).to(DEV)
        jobs.append((_params(mods, D, k), smp, perm))

    def run(concurrent, use_ws):
        outs, streams, keep = [], [torch.cuda.Stream(DEV), torch.cuda.Stream(DEV)], []
        torch.cuda.synchronize()
        for k, (p0, smp, perm) in enumerate(jobs):
            p = p0.clone()
            m, v = torch.zeros_like(p), torch.zeros_like(p)
            st = torch.zeros((), device=DEV)
            sums = torch.zeros(4, dtype=torch.float64, device=DEV)
            ws = torch.zeros(int(lib.ppo_workspace_bytes()), dtype=torch.uint8, device=DEV)
            hp = _hp(L, cfg)
            s = streams[k] if concurrent else torch.cuda.current_stream(DEV)
            s.wait_stream(torch.cuda.current_stream(DEV))
            args = [L.ptr(p), L.ptr(m), L.ptr(v), L.ptr(st), D] + [L.ptr(t) for t in smp] + \
                   [n, L.ptr(perm), E, 64, ctypes.byref(hp), L.ptr(sums)]
            sp = ctypes.c_void_p(s.cuda_stream)
            if use_ws:
                L.check(lib.ppo_update_ws(*args, L.ptr(ws), sp), "ppo_update_ws")
            else:
                L.check(lib.ppo_update(*args, sp), "ppo_update")
            keep.append(hp)
            outs.append((p, m, v, st, sums))
        torch.cuda.synchronize()
        return outs

    serial = run(False, True)
    for use_ws in (True, False):
        conc = run(True, use_ws)
        for a, b in zip(serial, conc):
            for x, y in zip(a, b):
                assert torch.equal(x, y), use_ws
    for _, _, _, _, sums in serial:
        s = sums.tolist()
        assert not math.isnan(s[0]) and s[3] >= 0  # no lost exchange


@pytest.mark.parametrize("D", [8, 6])
def test_ppo_grad_matches_autograd(mods, D):
    """ppo_grad (the fused kernel in gradient mode) == torch autograd of the same rank-local loss
    share (dp_update.ShardedUpdate._local_grad_eager): b_local = 24 of b_global = 64 samples,
    global advantage statistics, the entropy term on (rank 0) and off; fp32 summation order and
    the kernel's exp/rcp tanh (< 3e-7 absolute) are the only differences."""
    L = mods["_lib"]
    cfg = mods["ppo"].PPOConfig(batch_size=64, update_mode="sharded")
    smp = list(_samples(300, D, 3))
    smp[4] = smp[4] * 135.0  # returns at the reference config's scale (value loss ~1.8e4)
    flat = _params(mods, D, 1)
    rows = torch.randperm(300, generator=torch.Generator().manual_seed(4))[:24].to(DEV)
    for ent_once in (1, 0):
        upd = mods["dp_update"].ShardedUpdate(cfg, D, [300], 0, DEV)
        upd.rank = 0 if ent_once else 1
        param = torch.nn.Parameter(flat.clone())
        upd._local_grad_eager(param, smp, rows, 64, 0.3, 1.7)
        want, want_sums = param.grad.clone(), upd.sums.clone()
        grad = torch.full_like(flat, 7.0)
        sums = torch.zeros(4, dtype=torch.float64, device=DEV)
        hp = _hp(L, cfg)
        L.check(L.lib().ppo_grad(L.ptr(flat), D, *(L.ptr(t) for t in smp), L.ptr(rows), 24, 64,
                                 0.3, 1.7, 1, ent_once, ctypes.byref(hp), L.ptr(grad),
                                 L.ptr(sums), L.current_stream(DEV)), "ppo_grad")
        torch.cuda.synchronize()
        scale = want.abs().max().item()
        err = (grad - want).abs().max().item()
        assert err <= 2e-6 * scale, (ent_once, err, scale)
        # per parameter group too: the value head's gradient (large returns) must not hide an
        # error in a small group such as log_std
        for name, (a, b) in _groups(D).items():
            gs = want[a:b].abs().max().item()
            ge = (grad[a:b] - want[a:b]).abs().max().item()
            print(f"grad group {name:8s} D={D} ent_once={ent_once} max|g| {gs:.3e} err {ge:.3e}")
            assert ge <= 1e-5 * gs + 1e-9, (name, ge, gs)
        torch.testing.assert_close(sums, want_sums, rtol=1e-5, atol=1e-7)
    # no rows on this rank: a zero gradient (+ the entropy term where it lives)
    grad = torch.full_like(flat, 7.0)
    L.check(L.lib().ppo_grad(L.ptr(flat), D, *(L.ptr(t) for t in smp), None, 0, 64, 0.0, 1.0, 1,
                             1, ctypes.byref(_hp(L, cfg)), L.ptr(grad), L.ptr(sums),
                             L.current_stream(DEV)), "ppo_grad")
    torch.cuda.synchronize()
    assert torch.equal(grad[:-2], torch.zeros_like(grad[:-2]))
    assert torch.equal(grad[-2:], torch.full((2,), -cfg.ent_coef, device=DEV))


def test_ppo_grad_tiny_dz2_not_flushed(mods):
    """the W2-gradient phase scales dL/dz2 by the power of two that puts its largest
    entry at 2^10..2^11 for the split-f16 MFMAs and multiplies the results back.  With max
    |dL/dz2| below 2^-116 the clamped scale exponent made the unscale factor +0.0 and zeroed the
    W2 and dL/dh1 gradients (csrc/ppo_update.hip, W2 phase).  Here advantages ~1e-34 (no
    normalisation) and vf_coef 1e-34 put max |dL/dz2| near 1e-37 on both networks: every parameter
    group's gradient must equal autograd's at the usual relative bound, and none may be zero."""
    L = mods["_lib"]
    D = 8
    cfg = mods["ppo"].PPOConfig(batch_size=64, update_mode="sharded", normalize_advantage=False,
                                vf_coef=1e-34)
    obs, act, lp, adv, ret = _samples(300, D, 5)
    smp = [obs, act, lp, adv * 1e-34, ret]
    flat = _params(mods, D, 2)
    rows = torch.randperm(300, generator=torch.Generator().manual_seed(6))[:64].to(DEV)
    upd = mods["dp_update"].ShardedUpdate(cfg, D, [300], 0, DEV)
    upd.rank = 1  # no entropy term: it does not pass through dL/dz2 and would swamp log_std
    param = torch.nn.Parameter(flat.clone())
    upd._local_grad_eager(param, smp, rows, 64, 0.0, 1.0)
    want = param.grad.clone()
    grad = torch.full_like(flat, 7.0)
    sums = torch.zeros(4, dtype=torch.float64, device=DEV)
    hp = _hp(L, cfg)
    hp.normalize_advantage = 0
    L.check(L.lib().ppo_grad(L.ptr(flat), D, *(L.ptr(t) for t in smp), L.ptr(rows), 64, 64, 0.0,
                             1.0, 0, 0, ctypes.byref(hp), L.ptr(grad), L.ptr(sums),
                             L.current_stream(DEV)), "ppo_grad")
    torch.cuda.synchronize()
    for name, (a, b) in _groups(D).items():
        if name == "log_std":
            continue  # ~1e-33 from the policy term alone; compared below with the rest
        gs = want[a:b].abs().max().item()
        ge = (grad[a:b] - want[a:b]).abs().max().item()
        print(f"tiny grad group {name:8s} max|g| {gs:.3e} err {ge:.3e}")
        assert 0.0 < gs < 1e-30, (name, gs)
        assert grad[a:b].abs().max().item() > 0.0, name
        assert ge <= 1e-5 * gs, (name, ge, gs)


def test_ppo_apply_matches_torch_adam(mods):
    """ppo_apply == torch clip_grad_norm_ + Adam(capturable) over 20 steps from the same
    gradients (one clipped, one not, per step)."""
    L = mods["_lib"]
    cfg = mods["ppo"].PPOConfig()
    flat = _params(mods, 8, 2)
    param = torch.nn.Parameter(flat.clone())
    opt = torch.optim.Adam([param], lr=1e-3, eps=1e-5, capturable=True)
    p, m, v = flat.clone(), torch.zeros_like(flat), torch.zeros_like(flat)
    st = torch.zeros((), device=DEV)
    g = torch.Generator().manual_seed(9)
    hp = _hp(L, cfg)
    for k in range(20):
        grad = (torch.randn(flat.shape, generator=g) * (0.001 if k % 2 else 0.05)).to(DEV)
        param.grad = grad.clone()
        torch.nn.utils.clip_grad_norm_([param], cfg.max_grad_norm)
        opt.step()
        L.check(L.lib().ppo_apply(L.ptr(p), L.ptr(m), L.ptr(v), L.ptr(st), L.ptr(grad), 8,
                                  ctypes.byref(hp), L.current_stream(DEV)), "ppo_apply")
    torch.cuda.synchronize()
    s = opt.state[param]
    assert float(st) == float(s["step"]) == 20.0
    # (1 - beta) is formed from the fp32 hyper-parameters in the kernel: float32(1 - 0.999f) is
    # 1.29e-5 relative below torch's float32(0.001) (a Python double), so exp_avg_sq's increments
    # differ by that factor (2e-5 bound), exp_avg's by 2.4e-7, and the steps by ~6.5e-6 relative
    torch.testing.assert_close(m, s["exp_avg"], rtol=1e-5, atol=1e-9)
    torch.testing.assert_close(v, s["exp_avg_sq"], rtol=2e-5, atol=1e-12)
    moved = (param.detach() - flat).abs().max().item()
    assert moved > 1e-3
    assert (p - param.detach()).abs().max().item() <= 3e-5 * moved


def test_sharded_update_fused_equals_eager(mods):
    """The data-parallel update on one rank (dp_update.ShardedUpdate.run): fused kernels
    (ppo_grad + ppo_apply per minibatch) == torch autograd + torch Adam, 3 epochs over 1,000
    samples in minibatches of 64 (the last one 40)."""
    cfg = mods["ppo"].PPOConfig(n_epochs=3, update_mode="sharded")
    smp = _samples(1000, 8, 5)
    flat = _params(mods, 8, 3)
    outs = []
    for fused in (False, True):
        param = torch.nn.Parameter(flat.clone())
        opt = torch.optim.Adam([param], lr=1e-3, eps=1e-5, capturable=True)
        upd = mods["dp_update"].ShardedUpdate(cfg, 8, [1000], 7, DEV, fused=fused)
        stats = upd.run(param, opt, smp)
        outs.append((param.detach().clone(), stats))
    (p0, s0), (p1, s1) = outs
    moved = (p0 - flat).abs().max().item()
    err = (p1 - p0).abs().max().item()
    assert moved > 1e-2 and err <= 1e-4 * moved, (moved, err)
    for k in s0:
        assert abs(s0[k] - s1[k]) <= 1e-4 * max(1.0, abs(s0[k])), (k, s0[k], s1[k])


def test_fused_update_vs_torch_at_reference_config(mods):
    """One full PPO update at the reference's training configuration
    (/root/reference/vectorized_env.py:126-131: 1,000 formations x 5 agents, n_steps 10,
    batch 64, 10 epochs = 7,820 dependent minibatches): the fused kernel (ppo_update) against
    torch autograd + torch Adam (the eager minibatch step, replayed as a HIP graph) on the same
    samples and permutations.

    A 7,820-step trajectory of the clipped surrogate is not a smooth function of its inputs (a
    sample whose probability ratio sits at 1 +- clip_range, or a torch.min tie, flips its gradient
    for a last-bit difference, and Adam carries it forward), so the reference spread is torch
    itself started ONE ulp away (every parameter moved up by one ulp); the fused update may be 3x
    as far from torch as that run is, plus
    * for the parameters, a coherent part K * lr * delta = 7,820 * 1e-3 * 4e-6 (delta = twice the
      per-minibatch gradient agreement test_ppo_grad_matches_autograd measures);
    * for every loss mean, 1e-5 relative (the north star's fp32 bound).
    Round 4: the kernel's Adam used 1 - fp32(beta) for the moment rates where torch
    uses fp32(1 - beta) formed in double (1.3e-5 relative apart for beta2 = 0.999, a coherent bias
    of every second moment) and exp2f(step * log2f(beta)) for beta^step (up to 1 ulp off); with
    torch's forms the update lands 2-200x closer to torch (profiles/ab/r4_ppo_precision_ab.txt), and
    test_fused_step_unbiased_along_reference_trajectory checks each step against float64."""
    cfg = {"num_formation": 1000, "num_agents_per_formation": 5, "goal_in_obs": True}

    def run(fused, ulp):
        env = mods["vectorized_env"].FormationEnv(cfg, device=DEV, seed=2, reset_mode="philox")
        ppo = mods["ppo"].PPO(env, mods["ppo"].PPOConfig(), seed=3, use_graph=not fused,
                              use_fused=fused)
        with torch.no_grad():
            ppo.collector.collect()  # the rollout uses the unperturbed parameters
            if ulp:  # one ulp up (nextafter: zeros move to the smallest subnormal)
                f = ppo.policy.flat
                f.copy_(torch.nextafter(f, torch.full_like(f, math.inf)))
        flat0 = ppo.policy.flat.clone()
        st = ppo.train()
        s = ppo.opt.state[ppo.param]
        assert float(s["step"]) == 7820
        env.release()
        return flat0, ppo.policy.flat.clone(), st

    a0, p0, s0 = run(False, False)
    _, pu, su = run(False, True)
    a1, p1, s1 = run(True, False)
    assert torch.equal(a0, a1)
    moved = (p0 - a0).abs()
    d_fused, d_ulp = (p1 - p0).abs(), (pu - p0).abs()
    print(f"\nreference-config update: max moved {moved.max().item():.4g}; |fused - torch| max "
          f"{d_fused.max().item():.3g} median {d_fused.median().item():.3g}; |torch(1 ulp) - "
          f"torch| max {d_ulp.max().item():.3g} median {d_ulp.median().item():.3g}")
    print(f"losses torch {s0}\n       fused {s1}\n  torch 1ulp {su}")
    coherent = 7820 * 1e-3 * 4e-6
    assert moved.max().item() > 0.1  # the update did move the parameters
    assert d_fused.max().item() <= 3 * d_ulp.max().item() + coherent
    assert d_fused.median().item() <= 3 * d_ulp.median().item() + coherent
    # The three continuous loss means are held to the north star's plain fp32 bound, with no
    # allowance for torch's own 1-ulp spread (round 4's last run: policy_gradient_loss 4.6e-6
    # apart, value_loss 1.6e-4 of 18,306, entropy_loss 5.4e-6 of 2.83).
    for k in ("policy_gradient_loss", "value_loss", "entropy_loss"):
        assert abs(s1[k] - s0[k]) <= 1e-5 * max(1.0, abs(s0[k])), (k, s0[k], s1[k], su[k])
    # clip_fraction counts samples whose ratio left [1 - 0.2, 1 + 0.2]: a discrete mean, one
    # sample flipping moves it by 1 / (64 * 7,820) = 2.0e-6, and which samples sit on the edge is
    # exactly what a last-bit difference decides.  Torch moved one ulp is 2.8e-5 (14 samples)
    # from torch, the fused kernel 1.6e-5 (8 samples) -- over the plain 1e-5, so this mean alone
    # keeps the chaotic term: within 3x torch's own 1-ulp spread, plus 1e-5.
    k = "clip_fraction"
    assert abs(s1[k] - s0[k]) <= 3 * abs(su[k] - s0[k]) + 1e-5, (k, s0[k], s1[k], su[k])
    assert set(s0) == {"policy_gradient_loss", "value_loss", "entropy_loss", "clip_fraction"}


def test_fused_step_unbiased_along_reference_trajectory(mods, flib):
    """no systematic error in the fused update's step.  Along the first 1,000
    minibatches of the reference-config trajectory (torch's), each minibatch's update is computed
    from torch's own parameters and Adam state three ways -- float64 (autograd, clip_grad_norm_,
    Adam with torch's formulas: the truth), torch fp32, and the fused kernel (ppo_update_ws over that
    minibatch alone) -- and per parameter group (log_std included) the signed relative step error
    against float64 must be as unbiased as torch fp32's (means within 3 standard errors + 1e-6)
    and no noisier than 1.2x torch's (tools/ppo_step_probe.py runs the whole trajectory:
    profiles/r4_ppo_step_probe.json)."""
    import ctypes
    L = mods["_lib"]
    ppo_mod = mods["ppo"]
    env = mods["vectorized_env"].FormationEnv(
        {"num_formation": 1000, "num_agents_per_formation": 5, "goal_in_obs": True}, device=DEV,
        seed=2, reset_mode="philox")
    m = ppo_mod.PPO(env, ppo_mod.PPOConfig(), seed=3, use_graph=False, use_fused=False)
    c = m.cfg
    with torch.no_grad():
        m.collector.collect()
    obs, act, old_lp, adv, ret = (t.contiguous() for t in m._flat())
    n, D = obs.shape
    perm = ppo_mod.epoch_permutations(n, c.n_epochs, torch.Generator(device=DEV).manual_seed(3),
                                      DEV)
    B1, B2, EPS, LR = 0.9, 0.999, 1e-5, c.learning_rate
    hp = L.PPOHParams(clip_range=c.clip_range, ent_coef=c.ent_coef, vf_coef=c.vf_coef,
                      max_grad_norm=c.max_grad_norm, lr=LR, beta1=B1, beta2=B2, eps=EPS,
                      normalize_advantage=1)
    lib = L.lib()
    ws = torch.zeros(int(lib.ppo_workspace_bytes()), dtype=torch.uint8, device=DEV)
    stats = torch.zeros(4, dtype=torch.float64, device=DEV)
    groups, o = [], 0
    for k, shp in m.policy.param_shapes():
        groups.append((k, o, o + math.prod(shp)))
        o += math.prod(shp)

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
    acc = {w: torch.zeros((3, G), dtype=torch.float64, device=DEV) for w in ("k", "t")}
    for kmb in range(1000):
        e, s0_ = divmod(kmb, -(-n // c.batch_size))
        idx = perm[e, s0_ * c.batch_size:(s0_ + 1) * c.batch_size].contiguous()
        B = idx.numel()
        st = opt.state[param]
        if st:
            mk, vk, sk = st["exp_avg"].clone(), st["exp_avg_sq"].clone(), st["step"].clone()
        else:
            mk, vk = torch.zeros_like(param), torch.zeros_like(param)
            sk = torch.zeros((), dtype=torch.float32, device=DEV)
        p0 = param.detach().clone()
        g64 = grad(param, idx, torch.float64)
        g64 = g64 * min(1.0, c.max_grad_norm / (g64.norm().item() + 1e-6))
        t = kmb + 1
        ms, vs = mk.double(), vk.double()
        m_n = ms + (1 - B1) * (g64 - ms)
        v_n = vs * B2 + (1 - B2) * g64 * g64
        d64 = -(LR / (1 - B1 ** t)) * m_n / (v_n.sqrt() / math.sqrt(1 - B2 ** t) + EPS)
        rows = [x[idx].contiguous() for x in (obs, act, old_lp, adv, ret)]
        pk = p0.clone()
        ar = torch.arange(B, device=DEV, dtype=torch.long)
        flib.check(lib.ppo_update_ws(L.ptr(pk), L.ptr(mk), L.ptr(vk), L.ptr(sk), D,
                                     *(L.ptr(x) for x in rows), B, L.ptr(ar), 1, B,
                                     ctypes.byref(hp), L.ptr(stats), L.ptr(ws),
                                     L.current_stream(torch.device(DEV))), "ppo_update_ws")
        param.grad = grad(param, idx, torch.float32)
        torch.nn.utils.clip_grad_norm_([param], c.max_grad_norm)
        opt.step()
        sel = d64.abs() > 1e-3 * LR
        for w, d in (("k", (pk - p0).double()), ("t", (param.detach() - p0).double())):
            r = torch.where(sel, (d - d64) * torch.sign(d64) / d64.abs().clamp(min=1e-30), 0.0)
            for gi, (_, lo, hi) in enumerate(groups):
                acc[w][0, gi] += r[lo:hi].sum()
                acc[w][1, gi] += r[lo:hi].pow(2).sum()
                acc[w][2, gi] += sel[lo:hi].sum()
    env.release()
    for gi, (name, _, _) in enumerate(groups):
        cnt = max(1.0, acc["k"][2, gi].item())
        mk_, mt_ = acc["k"][0, gi].item() / cnt, acc["t"][0, gi].item() / cnt
        rk, rt = (math.sqrt(acc[w][1, gi].item() / cnt) for w in ("k", "t"))
        assert abs(mk_ - mt_) <= 3 * (rk + rt) / math.sqrt(cnt) + 1e-6, (name, mk_, mt_, rk, rt)
        assert rk <= 1.2 * rt + 1e-6, (name, rk, rt)


def test_ppo_sharded_mode_trains(mods):
    """PPO(update_mode="sharded") on one rank: collect + train through the fused ppo_grad /
    ppo_apply kernels; finite losses, the Adam step count of 2 updates x 3 epochs x 4 minibatches."""
    env = mods["vectorized_env"].FormationEnv(
        {"num_formation": 40, "num_agents_per_formation": 5, "goal_in_obs": True}, device=DEV,
        seed=1, reset_mode="philox")
    ppo = mods["ppo"].PPO(env, mods["ppo"].PPOConfig(n_epochs=3, batch_size=512,
                                                     update_mode="sharded"), seed=2)
    assert ppo._dp is not None and ppo._dp.fused is False  # batch 512 > 64: the torch path
    ppo2 = mods["ppo"].PPO(env, mods["ppo"].PPOConfig(n_epochs=3, batch_size=64,
                                                      update_mode="sharded"), seed=2)
    assert ppo2._dp.fused
    for p in (ppo, ppo2):
        for _ in range(2):
            with torch.no_grad():
                p.collector.collect()
            st = p.train()
            assert all(math.isfinite(v) for v in st.values()), st
    assert float(ppo.opt.state[ppo.param]["step"]) == 2 * 3 * 4
    assert float(ppo2.opt.state[ppo2.param]["step"]) == 2 * 3 * 32
    env.release()


def test_lost_exchange_rerun_and_raise(mods, flib):
    """The fused update's lost-exchange paths (nothing forced them).  With the test hook
    fenv_test_ppo_inject(1) the first launch loses its norm exchange: ppo.py sees the marked stats,
    restores the pre-launch state and runs again, and the result equals a clean update bit for bit
    (the kernel is deterministic).  With two lost launches it raises and leaves the pre-update
    parameters and Adam state in place."""
    cfg = {"num_formation": 100, "num_agents_per_formation": 5, "goal_in_obs": True}
    outs = []
    for inject in (0, 1, 2):
        env = mods["vectorized_env"].FormationEnv(cfg, device=DEV, seed=2, reset_mode="philox")
        ppo = mods["ppo"].PPO(env, mods["ppo"].PPOConfig(n_epochs=2), seed=3, use_fused=True)
        with torch.no_grad():
            ppo.collector.collect()
        ppo.train()
        with torch.no_grad():
            ppo.collector.collect()
        st = ppo.opt.state[ppo.param]
        before = tuple(t.detach().clone() for t in (ppo.param, st["exp_avg"], st["exp_avg_sq"],
                                                    st["step"]))
        flib.lib().fenv_test_ppo_inject(inject)
        try:
            if inject == 2:
                with pytest.raises(RuntimeError, match="exchange timed out twice"):
                    ppo.train()
                after = (ppo.param, st["exp_avg"], st["exp_avg_sq"], st["step"])
                for a, b in zip(before, after):
                    assert torch.equal(a, b)
            else:
                stats = ppo.train()
                assert ppo.exchange_retries == inject
                outs.append((ppo.param.detach().clone(), st["exp_avg_sq"].clone(), stats))
        finally:
            flib.lib().fenv_test_ppo_inject(0)
        env.release()
    (p0, v0, s0), (p1, v1, s1) = outs
    assert torch.equal(p0, p1) and torch.equal(v0, v1) and s0 == s1
