"""GPU parity at BASELINE.json's full sizes (configs 1-4: 4,096 x 5, 65,536 x 10, 1,048,576 x 5,
16,384 x 64), where the CPU oracle cannot replay the whole batch in seconds.

Formations are independent (no cross-formation term in simulate.py:150-236), so a sample of
formations -- random ones plus the first and last two, i.e. the grid's first wavefront and its
partial last one -- is replayed by the C oracle from the GPU's own state and actions and must
match bit for bit over a fused 10-step rollout (the bench's launch).  Size-independent checks
cover the rest of the arrays: the per-workgroup {reward, done} records reduce to the sums of the
full reward/done arrays (checksum of checksums), the last observation is the final state
normalised (simulate.py:156-160) for every agent, and no agent moved more than 10 px per axis per
step (vectorized_env.py:69-70 with |a| <= 1.2)."""
import numpy as np
import pytest
import torch

from oracle import COracleEnv
from tolerance import assert_rel_close

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
T = 10


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint32) if a.dtype == np.float32 else a


@pytest.mark.parametrize("F,N,goal", [(4096, 5, True), (65536, 10, True), (1 << 20, 5, True),
                                      (1 << 20, 5, False), (16384, 64, True)])
def test_full_size_sampled_vs_oracle(venv, F, N, goal):
    env = venv.FormationEnv({"num_formation": F, "num_agents_per_formation": N,
                             "goal_in_obs": goal}, device=DEV, seed=21, reset_mode="philox")
    A, D = F * N, env.obs_dim
    env.reset_tensor()
    g = torch.Generator(device=DEV).manual_seed(F + N)
    env.rollout(torch.rand((T, A, 2), device=DEV, generator=g) * 2.4 - 1.2)  # varied state, t > 0
    px0, py0, gx0, gy0, t0 = env.get_state()
    acts = torch.rand((T, A, 2), device=DEV, generator=g) * 2.4 - 1.2
    part = torch.zeros((env.partial_count(), 2), dtype=torch.float32, device=DEV)
    obs, rew, done = env.rollout(acts, partial=part)
    sums = env.reduce_partials(part).cpu().numpy()
    px1, py1, gx1, gy1, t1 = env.get_state()
    torch.cuda.synchronize()

    rng = np.random.default_rng(F * 131 + N)
    fs = np.unique(np.concatenate([rng.choice(F, min(F, 3000), replace=False),
                                   [0, 1, F - 2, F - 1]]))
    ag = (fs[:, None] * N + np.arange(N)).reshape(-1)
    agt, fst = torch.from_numpy(ag).to(DEV), torch.from_numpy(fs).to(DEV)
    ref = COracleEnv(len(fs), N, goal, 0)
    ref.set_state(*(v[agt].cpu().numpy() for v in (px0, py0)),
                  *(v[fst].cpu().numpy() for v in (gx0, gy0, t0)))
    a_s = acts[:, agt].cpu().numpy()
    o_s, r_s, d_s = obs[:, agt].cpu().numpy(), rew[:, agt].cpu().numpy(), done[:, agt].cpu().numpy()
    for j in range(T):
        ro, rr, rd, _ = ref.step(np.ascontiguousarray(a_s[j]))
        assert np.array_equal(bits(o_s[j]), bits(ro)), f"obs step {j}"
        assert np.array_equal(bits(r_s[j]), bits(rr)), f"reward step {j}"
        assert np.array_equal(d_s[j], rd), f"done step {j}"
    rs = ref.get_state()
    for name, v, w, idx in (("px", px1, rs[0], agt), ("py", py1, rs[1], agt),
                            ("gx", gx1, rs[2], fst), ("gy", gy1, rs[3], fst),
                            ("t", t1, rs[4], fst)):
        assert np.array_equal(bits(v[idx].cpu().numpy()), bits(w)), name

    # checksum of checksums: the stats records cover every agent-step exactly once
    rsum = rew.double().sum().item()
    assert abs(sums[0] - rsum) <= 1e-5 * max(1.0, abs(rsum)), (sums[0], rsum)
    assert sums[1] == float(done.sum().item())
    # the last observation is the final state, normalised, for every agent
    p1x, p1y = px1.cpu().numpy(), py1.cpu().numpy()
    last = obs[-1].cpu().numpy()
    assert np.array_equal(bits(last[:, 0]), bits(p1x / np.float32(400.0)))
    assert np.array_equal(bits(last[:, 1]), bits(p1y / np.float32(600.0)))
    if goal:
        gxa = np.repeat(gx1.cpu().numpy(), N)
        assert np.array_equal(bits(last[:, 6]), bits((gxa - p1x) / np.float32(400.0)))
    # kinematics bound and no timeout inside these 20 steps (episode = 1002 steps)
    p0x = px0.cpu().numpy()
    assert np.abs(p1x - p0x).max() <= 10 * 1.2 * T + 1e-3
    assert not done.any().item() and np.all(t1.cpu().numpy() == 2 * T)


def _normals(rows: np.ndarray, seed: int, offset: int) -> np.ndarray:
    """policy_oracle.philox_normals for selected rows (the kernel keys the noise by agent row)."""
    import math

    import policy_oracle as po
    r64 = rows.astype(np.uint64)
    ctr = np.stack([r64 & np.uint64(0xFFFFFFFF), r64 >> np.uint64(32),
                    np.full(len(rows), offset & 0xFFFFFFFF, np.uint64),
                    np.full(len(rows), (offset >> 32) & 0xFFFFFFFF, np.uint64)], axis=1)
    r = po._philox(ctr, (seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF))
    u1 = ((r[:, 0] >> np.uint64(8)) + np.uint64(1)).astype(np.float64) * 2.0 ** -24
    u2 = (r[:, 1] >> np.uint64(8)).astype(np.float64) * 2.0 ** -24
    rad = np.sqrt(-2.0 * np.log(u1))
    return np.stack([rad * np.cos(2 * math.pi * u2), rad * np.sin(2 * math.pi * u2)], axis=1)


def test_full_size_policy_rollout_sampled(pkg, venv):
    """BASELINE config 2 (65,536 formations x 10 agents) through the fused PPO collection kernel
    (fenv_policy_rollout: policy + Gaussian sample + clip + env step x 10, last value, GAE), a
    sample of formations checked against the CPU oracles: the policy (mu, value, action,
    log_prob, last value) against oracle/policy_oracle.py + the Philox noise restatement at the
    north star's 1e-5 relative (tests/tolerance.py), every env transition bit for bit against the
    C oracle, GAE against SB3's recurrence."""
    from importlib import import_module

    import policy_oracle as po
    ro = import_module(pkg.__name__ + ".rollout")
    pol_mod = import_module(pkg.__name__ + ".policy")
    F, N, D = 65536, 10, 8
    A = F * N
    env = venv.FormationEnv({"num_formation": F, "num_agents_per_formation": N,
                             "goal_in_obs": True}, device=DEV, seed=3, reset_mode="philox")
    pol = pol_mod.MlpPolicy(D, device=DEV, seed=2)
    with torch.no_grad():  # non-trivial heads so the actions move the agents
        pol.flat.add_(torch.randn(pol.flat.shape, generator=torch.Generator().manual_seed(5))
                      .to(DEV) * 0.05)
    buf = ro.RolloutBuffer(T, A, D, DEV)
    col = ro.RolloutCollector(env, pol, buf, seed=11, fused=True)
    col.collect()  # first rollout: states leave the reset distribution
    pre = [v.cpu().numpy() for v in env.get_state()]
    obs0 = col.last_obs.cpu().numpy()
    off0 = col.offset
    col.collect()
    torch.cuda.synchronize()

    rng = np.random.default_rng(17)
    fs = np.unique(np.concatenate([rng.choice(F, 2000, replace=False), [0, 1, F - 2, F - 1]]))
    ag = (fs[:, None] * N + np.arange(N)).reshape(-1)
    agt = torch.from_numpy(ag).to(DEV)
    S = len(ag)
    get = lambda t: t[:, agt].cpu()  # noqa: E731
    obs, mu, val = get(buf.observations), get(buf.mu), get(buf.values)
    act, clp, lp = get(buf.actions), get(buf.clipped), get(buf.log_probs)
    rew, dn, starts = get(buf.rewards), get(buf.dones), get(buf.episode_starts)
    adv, ret = get(buf.advantages), get(buf.returns)
    last_obs, last_val = col.last_obs[agt].cpu(), col._last_values[agt].cpu()
    assert np.array_equal(bits(obs[0].numpy()), bits(obs0[ag]))

    sd = po.unflatten(pol.flat.detach().cpu(), D)
    mu_ref, v_ref = po.forward(sd, obs.reshape(-1, D))
    assert_rel_close(mu.reshape(-1, 2), mu_ref, "mu")
    assert_rel_close(val.reshape(-1), v_ref, "value")
    std = sd["log_std"].exp().double()
    mu_ref = mu_ref.reshape(T, S, 2).double()
    for j in range(T):
        eps = torch.from_numpy(_normals(ag, 11, off0 + j))
        assert_rel_close(act[j], mu_ref[j] + std * eps, f"action step {j}")
    assert torch.equal(clp, act.clamp(-1, 1))
    assert_rel_close(lp.reshape(-1), po.log_prob({"log_std": sd["log_std"].double()},
                                                 mu_ref.reshape(-1, 2),
                                                 act.reshape(-1, 2).double()), "log_prob")
    _, lv_ref = po.forward(sd, last_obs)
    assert_rel_close(last_val, lv_ref, "last value")

    ref = COracleEnv(len(fs), N, True, 0)
    ref.set_state(pre[0][ag], pre[1][ag], pre[2][fs], pre[3][fs], pre[4][fs])
    for j in range(T):
        o, r, d, _ = ref.step(np.ascontiguousarray(clp[j].numpy()))
        nxt = obs[j + 1] if j + 1 < T else last_obs
        assert np.array_equal(bits(nxt.numpy()), bits(o)), f"obs step {j}"
        assert np.array_equal(bits(rew[j].numpy()), bits(r)), f"reward step {j}"
        assert np.array_equal(dn[j].numpy(), d), f"done step {j}"

    # GAE (SB3 RolloutBuffer.compute_returns_and_advantage), float64 recurrence
    g, lam = buf.gamma, buf.gae_lambda
    v64, r64 = val.double().numpy(), rew.double().numpy()
    nt = 1.0 - np.concatenate([starts[1:].numpy(), dn[-1:].numpy()]).astype(np.float64)
    nv = np.concatenate([v64[1:], last_val.double().numpy()[None]])
    gae = np.zeros(S)
    adv_ref = np.zeros((T, S))
    for j in reversed(range(T)):
        delta = r64[j] + g * nv[j] * nt[j] - v64[j]
        gae = delta + g * lam * nt[j] * gae
        adv_ref[j] = gae
    np.testing.assert_allclose(adv.numpy(), adv_ref, rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(ret.numpy(), adv_ref + v64, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("F,N,goal,T", [
    # 3e8 agents, D = 8: obs element offsets pass 2^31 and 2^32 inside row 0 (staged kernel, T=2)
    (60_000_000, 5, True, 2),
    # 2.2e9 agents: agent indices pass 2^31 (single-step launches take the plain wave kernel)
    (440_000_000, 5, False, 1)])
def test_beyond_int32_sizes_sampled_vs_oracle(venv, F, N, goal, T):
    """Maximum sizes: batches whose agent or obs-element indices overflow 32 bits (HBM holds
    them: ~40 GB and ~150 GB here).  In-kernel Philox actions (fenv_rollout_random), sampled
    formations -- incl. the ones straddling every 2^31 / 2^32 index boundary and the grid's last
    ones -- replayed by the C oracle bit for bit; the stats records sum to the full reward array."""
    from oracle import philox_actions
    env = venv.FormationEnv({"num_formation": F, "num_agents_per_formation": N,
                             "goal_in_obs": goal}, device=DEV, seed=5, reset_mode="philox")
    A, D = F * N, env.obs_dim
    assert A * D > 1 << 31
    env.reset_tensor()
    px0, py0, gx0, gy0, t0 = env.get_state()
    rng = np.random.default_rng(F)
    edges = [(1 << 31) // (N * D), (1 << 32) // (N * D), (1 << 31) // N, (1 << 32) // N]
    fs = [rng.choice(F, 1500, replace=False), [0, 1, F - 2, F - 1]]
    fs += [[e - 1, e, e + 1] for e in edges if e + 1 < F]
    fs = np.unique(np.concatenate(fs)).astype(np.int64)
    ag = (fs[:, None] * N + np.arange(N)).reshape(-1)
    agt, fst = torch.from_numpy(ag).to(DEV), torch.from_numpy(fs).to(DEV)
    ref = COracleEnv(len(fs), N, goal, 0)
    ref.set_state(*(v[agt].cpu().numpy() for v in (px0, py0)),
                  *(v[fst].cpu().numpy() for v in (gx0, gy0, t0)))
    del px0, py0, gx0, gy0, t0
    part = torch.zeros((env.partial_count(), 2), dtype=torch.float32, device=DEV)
    seed = 91
    if T == 1:  # reuse the env's own [A, D] / [A] buffers (memory)
        obs, rew, done = env.rollout_random(1, seed, 0, obs=env.obs_dev.view(1, A, D),
                                            rew=env.rew_dev.view(1, A),
                                            done=env.done_dev.view(1, A), partial=part)
    else:
        obs, rew, done = env.rollout_random(T, seed, 0, partial=part)
    sums = env.reduce_partials(part).cpu().numpy()
    torch.cuda.synchronize()
    o_s, r_s, d_s = obs[:, agt].cpu().numpy(), rew[:, agt].cpu().numpy(), done[:, agt].cpu().numpy()
    for j in range(T):
        a_j = np.concatenate([philox_actions(seed, j, int(f) * N, N) for f in fs])
        ro, rr, rd, _ = ref.step(a_j)
        assert np.array_equal(bits(o_s[j]), bits(ro)), f"obs step {j}"
        assert np.array_equal(bits(r_s[j]), bits(rr)), f"reward step {j}"
        assert np.array_equal(d_s[j], rd), f"done step {j}"
    rs = ref.get_state()
    px1, py1, gx1, gy1, t1 = env.get_state()
    for name, v, w, idx in (("px", px1, rs[0], agt), ("py", py1, rs[1], agt),
                            ("gx", gx1, rs[2], fst), ("gy", gy1, rs[3], fst),
                            ("t", t1, rs[4], fst)):
        assert np.array_equal(bits(v[idx].cpu().numpy()), bits(w)), name
    rsum = rew.double().sum().item()
    assert abs(sums[0] - rsum) <= 1e-5 * max(1.0, abs(rsum)), (sums[0], rsum)
    assert sums[1] == 0.0 and not bool(done.any())
    assert bool((t1 == T).all())


def test_bench_workload_staggered_resets_vs_oracle(venv):
    """the benchmark's own workload -- BASELINE config 3 (1,048,576 x 5),
    Philox resets, episode phases staggered by bench.stagger_episodes (formation f starts at
    steps_since_reset f mod 1002, so 1/1002 of the formations reset at every step), one fused
    10-step launch (k_rollout_wave_rs with non-temporal stores, as timed) -- replayed across the
    resets.  The sample holds, for every step index j of the launch, formations that reset at j,
    plus random ones and the grid's ends.  The C oracle steps the GPU's pre-launch state: the
    done step's reward and done (scored on the pre-reset state) bit for bit; then the reset
    formations take oracle.philox_reset_draws (episode 3: ctor 1, reset() 2) and the post-reset
    observation, and every later step, must match bit for bit; the final state too."""
    import bench
    from oracle import philox_reset_draws
    F, N, T, ep_len = 1 << 20, 5, 10, 1002
    seed = 0
    env = venv.FormationEnv({"num_formation": F, "num_agents_per_formation": N,
                             "goal_in_obs": True}, device=DEV, seed=seed, reset_mode="philox")
    A = F * N
    env.reset_tensor()
    bench.stagger_episodes(env, 0)
    px0, py0, gx0, gy0, t0 = env.get_state()
    assert env.rollout_kernel_name(T) == "k_rollout_wave_rs"
    g = torch.Generator(device=DEV).manual_seed(1234)
    acts = torch.rand((T, A, 2), device=DEV, generator=g) * 2 - 1  # bench.py's action stream
    part = torch.zeros((env.partial_count(), 2), dtype=torch.float32, device=DEV)
    obs, rew, done = env.rollout(acts, partial=part)
    sums = env.reduce_partials(part).cpu().numpy()
    px1, py1, gx1, gy1, t1 = env.get_state()
    torch.cuda.synchronize()

    rng = np.random.default_rng(5)
    resetting = []
    for j in range(T):  # formations whose pre-step t at step j is max_steps + 1 = 1001
        cand = np.arange((ep_len - 1 - j) % ep_len, F, ep_len)
        resetting.append(rng.choice(cand, 40, replace=False))
    fs = np.unique(np.concatenate(resetting + [rng.choice(F, 1500, replace=False),
                                               [0, 1, F - 2, F - 1]]))
    ag = (fs[:, None] * N + np.arange(N)).reshape(-1)
    agt, fst = torch.from_numpy(ag).to(DEV), torch.from_numpy(fs).to(DEV)
    ref = COracleEnv(len(fs), N, True, 0)
    st = [px0[agt].cpu().numpy(), py0[agt].cpu().numpy(), gx0[fst].cpu().numpy(),
          gy0[fst].cpu().numpy(), t0[fst].cpu().numpy()]
    ref.set_state(*st)
    a_s = acts[:, agt].cpu().numpy()
    o_s, r_s, d_s = obs[:, agt].cpu().numpy(), rew[:, agt].cpu().numpy(), done[:, agt].cpu().numpy()
    seen = set()
    for j in range(T):
        _, rr, rd, _ = ref.step(np.ascontiguousarray(a_s[j]))
        assert np.array_equal(bits(r_s[j]), bits(rr)), f"reward step {j}"
        assert np.array_equal(d_s[j], rd), f"done step {j}"
        dfm = np.nonzero(rd.reshape(-1, N)[:, 0])[0]  # sample-local formations reset at j
        assert set(resetting[j]) <= set(fs[dfm].tolist()), f"expected resets missing at step {j}"
        seen.add(j)
        if dfm.size:  # the oracle drew from its MT19937 stream: put the Philox draw in place
            px, py, gx, gy, t = ref.get_state()
            rx, ry, rgx, rgy = philox_reset_draws(seed, fs[dfm], N, np.full(dfm.size, 3))
            ai = (dfm[:, None] * N + np.arange(N)).reshape(-1)
            px[ai], py[ai], gx[dfm], gy[dfm] = rx, ry, rgx, rgy
            assert np.all(t[dfm] == 0)
            ref.set_state(px, py, gx, gy, t)
        ro = ref.observe()
        assert np.array_equal(bits(o_s[j]), bits(ro)), f"obs step {j} (post-reset)"
    assert seen == set(range(T))
    rs = ref.get_state()
    for name, v, w, idx in (("px", px1, rs[0], agt), ("py", py1, rs[1], agt),
                            ("gx", gx1, rs[2], fst), ("gy", gy1, rs[3], fst),
                            ("t", t1, rs[4], fst)):
        assert np.array_equal(bits(v[idx].cpu().numpy()), bits(w)), name
    # size-independent: every formation reset exactly once in the window iff its phase says so,
    # and the stats records cover every agent-step
    tt0 = t0.cpu().numpy().astype(np.int64)
    want = (tt0 >= ep_len - T)
    got = done.cpu().numpy().reshape(T, F, N)[:, :, 0].any(0)
    assert np.array_equal(want, got)
    assert int(done.sum().item()) == int(want.sum()) * N
    rsum = rew.double().sum().item()
    assert abs(sums[0] - rsum) <= 1e-5 * max(1.0, abs(rsum)), (sums[0], rsum)
    assert sums[1] == float(done.sum().item())


@pytest.mark.parametrize("F,N", [(1 << 20, 5), (65536, 10), (16384, 64)])
def test_mt19937_config3_resets_vs_stream(venv, F, N):
    """MT19937 reset mode (the reference's exact RNG) at BASELINE config 3
    (1,048,576 x 5), where each draw set is 12.6M MT19937 words drawn by the library's
    block-twisted generator on its draw-ahead thread, staged through the pinned pool and copied
    by k_stage_copy (fenv_api.cpp).  max_steps 7 (episodes of 9 steps) puts two reset events
    inside the two fused 10-step launches (steps 9 and 18; the library splits each launch
    there).  Sampled formations -- random ones, the grid's ends and both sides of every
    4,096-formation draw chunk -- are checked against numpy's MT19937 at their stream offsets
    (oracle.mt_reset_draws, not the library's own generator): the reset() state (set 1) and each
    post-reset state (sets 2, 3); the C oracle replays every step between, bit for bit: the done
    step's reward and done on the pre-reset state, the post-reset observation, the final state.
    Also at configs 2 and 4's shapes (65,536 x 10, 16,384 x 64: other draw-chunk widths, the
    N = 64 kernels)."""
    from oracle import mt_reset_draws
    T, ms, seed = 10, 7, 4242 + N
    ep = ms + 2
    env = venv.FormationEnv({"num_formation": F, "num_agents_per_formation": N,
                             "goal_in_obs": True}, device=DEV, seed=seed, reset_mode="mt19937",
                            max_steps=ms)
    A = F * N
    env.reset_tensor()
    px0, py0, gx0, gy0, t0 = env.get_state()
    g = torch.Generator(device=DEV).manual_seed(77)
    acts = [torch.rand((T, A, 2), device=DEV, generator=g) * 2.4 - 1.2 for _ in range(2)]
    out = [env.rollout(a) for a in acts]
    px1, py1, gx1, gy1, t1 = env.get_state()
    torch.cuda.synchronize()

    rng = np.random.default_rng(9)
    chunk = 49152 // (2 * N + 2)  # formations per draw chunk (fenv_api.cpp draw_formations)
    edges = np.arange(chunk, F, chunk)
    fs = np.unique(np.concatenate([rng.choice(F, 1500, replace=False), [0, 1, F - 2, F - 1],
                                   edges - 1, edges])).astype(np.int64)
    ag = (fs[:, None] * N + np.arange(N)).reshape(-1)
    agt, fst = torch.from_numpy(ag).to(DEV), torch.from_numpy(fs).to(DEV)
    want = mt_reset_draws(seed, [1, 2, 3], F, fs, N)
    st = [px0[agt].cpu().numpy(), py0[agt].cpu().numpy(), gx0[fst].cpu().numpy(),
          gy0[fst].cpu().numpy(), t0[fst].cpu().numpy()]
    for name, a, b in zip(("px", "py", "gx", "gy"), st[:4], want[1]):
        assert np.array_equal(bits(a), bits(b)), f"reset() state {name}"
    assert np.all(st[4] == 0)
    ref = COracleEnv(len(fs), N, True, 0, max_steps=ms)
    ref.set_state(*st)
    resets = 0
    for k in range(2 * T):
        la, j = divmod(k, T)
        obs, rew, done = out[la]
        a_s = acts[la][j, agt].cpu().numpy()
        _, rr, rd, _ = ref.step(np.ascontiguousarray(a_s))
        assert np.array_equal(bits(rew[j, agt].cpu().numpy()), bits(rr)), f"reward step {k + 1}"
        assert np.array_equal(done[j, agt].cpu().numpy(), rd), f"done step {k + 1}"
        if (k + 1) % ep == 0:  # every formation times out together (lock-step episodes)
            assert rd.all() and bool(done[j].all()), f"step {k + 1}"
            resets += 1
            px, py, gx, gy, t = ref.get_state()
            px, py, gx, gy = want[1 + resets]  # the oracle drew from its own sample-local stream
            assert np.all(t == 0)
            ref.set_state(px, py, gx, gy, t)
        else:
            assert not rd.any() and not bool(done[j].any()), f"step {k + 1}"
        ro = ref.observe()
        assert np.array_equal(bits(obs[j, agt].cpu().numpy()), bits(ro)), f"obs step {k + 1}"
    assert resets == 2
    rs = ref.get_state()
    for name, v, w, idx in (("px", px1, rs[0], agt), ("py", py1, rs[1], agt),
                            ("gx", gx1, rs[2], fst), ("gy", gy1, rs[3], fst),
                            ("t", t1, rs[4], fst)):
        assert np.array_equal(bits(v[idx].cpu().numpy()), bits(w)), name
    env.release()


@pytest.mark.parametrize("F,N", [(1_048_576, 5), (16_384, 64)])
def test_numpy_face_full_size_matches_device_face(venv, F, N):
    """BASELINE configs 3 and 4 through the numpy face, whose kernel reads the actions from and
    writes obs / reward / done to device-mapped host memory over PCIe (non-temporal stores at
    this size): bit-identical to the device face on a twin env, step by step, across a reset
    event (max_steps 2)."""
    cfg = {"num_formation": F, "num_agents_per_formation": N, "goal_in_obs": True}
    env = venv.FormationEnv(cfg, device=DEV, seed=5, reset_mode="philox", max_steps=2, log=False)
    twin = venv.FormationEnv(cfg, device=DEV, seed=5, reset_mode="philox", max_steps=2, log=False)
    A = F * N
    o = env.reset()
    assert np.array_equal(o.view(np.uint32), twin.reset_tensor().cpu().numpy().view(np.uint32))
    g = torch.Generator(device=DEV).manual_seed(5)
    dones = 0
    for k in range(5):
        a = torch.rand((A, 2), device=DEV, generator=g) * 2.4 - 1.2
        o, r, d, _ = env.step(a.cpu().numpy())
        to, tr, td = twin.step_tensor(a)
        dones += int(d.sum())
        assert np.array_equal(o.view(np.uint32), to.cpu().numpy().view(np.uint32)), k
        assert np.array_equal(r.view(np.uint32), tr.cpu().numpy().view(np.uint32)), k
        assert np.array_equal(d, td.cpu().numpy()), k
    assert dones == A  # max_steps 2: a 4-step episode, every formation done once in 5 steps
    env.release()
    twin.release()
