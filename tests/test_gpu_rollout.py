"""GPU: device rollout collection, GAE kernel and the on-device PPO update.

GAE is checked against a numpy restatement of SB3 RolloutBuffer.compute_returns_and_advantage
(parity unpinned vs SB3 itself, which is not installed); the rollout against step-by-step
policy + env calls; the training-side torch model against the HIP policy kernel."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from tolerance import assert_rel_close

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def mods(pkg):
    from importlib import import_module
    return {m: import_module(pkg.__name__ + "." + m)
            for m in ("rollout", "ppo", "policy", "vectorized_env", "_lib")}


def gae_numpy(rew, values, starts, last_values, last_dones, gamma, lam):
    T, A = rew.shape
    adv = np.zeros((T, A), np.float32)
    last = np.zeros(A, np.float32)
    for k in reversed(range(T)):
        if k == T - 1:
            nnt = 1.0 - last_dones.astype(np.float32)
            nv = last_values
        else:
            nnt = 1.0 - starts[k + 1].astype(np.float32)
            nv = values[k + 1]
        delta = rew[k] + np.float32(gamma) * nv * nnt - values[k]
        last = delta + np.float32(gamma) * np.float32(lam) * nnt * last
        adv[k] = last
    return adv, adv + values


def test_gae_kernel(mods):
    T, A = 10, 70001
    g = torch.Generator().manual_seed(0)
    buf = mods["rollout"].RolloutBuffer(T, A, 8, DEV)
    buf.rewards.copy_(torch.randn((T, A), generator=g))
    buf.values.copy_(torch.randn((T, A), generator=g))
    buf.episode_starts.copy_(torch.rand((T, A), generator=g) < 0.1)
    lv = torch.randn(A, generator=g)
    ld = torch.rand(A, generator=g) < 0.1
    buf.compute_returns_and_advantage(lv.to(DEV), ld.to(DEV))
    adv, ret = gae_numpy(buf.rewards.cpu().numpy(), buf.values.cpu().numpy(),
                         buf.episode_starts.cpu().numpy(), lv.numpy(), ld.numpy(), 0.99, 0.95)
    np.testing.assert_allclose(buf.advantages.cpu().numpy(), adv, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(buf.returns.cpu().numpy(), ret, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("F,N", [(300, 5), (2, 1500)])  # fused kernel / unfused (N > 64)
def test_collect_matches_stepwise(mods, F, N):
    cfg = {"num_formation": F, "num_agents_per_formation": N, "goal_in_obs": True}
    env1 = mods["vectorized_env"].FormationEnv(cfg, device=DEV, seed=3)
    env2 = mods["vectorized_env"].FormationEnv(cfg, device=DEV, seed=3)
    pol = mods["policy"].MlpPolicy(8, device=DEV, seed=5)
    buf = mods["rollout"].RolloutBuffer(6, F * N, 8, DEV)
    col = mods["rollout"].RolloutCollector(env1, pol, buf, seed=11)
    col.collect()
    obs = env2.reset_tensor().clone()
    starts = torch.ones(F * N, dtype=torch.bool, device=DEV)
    for k in range(6):
        assert torch.equal(buf.observations[k], obs)
        r = pol.forward(obs, seed=11, offset=k)
        assert torch.equal(buf.actions[k], r["action"])
        assert torch.equal(buf.log_probs[k], r["log_prob"])
        o, rw, d = env2.step_tensor(r["clipped"])
        assert torch.equal(buf.rewards[k], rw) and torch.equal(buf.dones[k], d)
        assert torch.equal(buf.episode_starts[k], starts)
        obs = o.clone()
        starts = d.clone()
    assert col.num_timesteps == 6 * F * N


def test_torch_model_matches_kernel(mods):
    """The differentiable restatement PPO trains must equal what the rollout kernel computes."""
    pol = mods["policy"].MlpPolicy(8, device=DEV, seed=2)
    obs = torch.rand((5000, 8), device=DEV) * 2 - 1
    r = pol.forward(obs, seed=1, offset=0)
    v, lp, ent = mods["ppo"].evaluate_actions(pol, pol.flat, obs, r["action"])
    assert_rel_close(r["value"], v, "value")
    assert_rel_close(r["log_prob"], lp, "log_prob")
    assert torch.allclose(ent, torch.full_like(ent, 2 * (0.5 + 0.5 * np.log(2 * np.pi))))


@pytest.mark.parametrize("batch_size,n_epochs", [(1024, 4), (64, 2)])  # graph / fused update
def test_ppo_learns(mods, batch_size, n_epochs):
    cfg = {"num_formation": 256, "num_agents_per_formation": 5, "goal_in_obs": True}
    env = mods["vectorized_env"].FormationEnv(cfg, device=DEV, seed=0, reset_mode="philox")
    ppo = mods["ppo"].PPO(env, mods["ppo"].PPOConfig(batch_size=batch_size, n_epochs=n_epochs),
                          seed=0)
    before = ppo.policy.flat.clone()
    rewards = []

    def cb(p):
        rewards.append(float(p.buffer.rewards.mean()))

    ppo.learn(total_timesteps=256 * 5 * 10 * 30, callback=cb)
    assert len(rewards) == 30
    assert not torch.equal(before, ppo.policy.flat)
    assert all(np.isfinite(v) for v in ppo.stats.values())
    # learning signal: the average reward of the last rollouts beats the first ones
    assert np.mean(rewards[-5:]) > np.mean(rewards[:5])


FIELDS = ("observations", "actions", "clipped", "mu", "values", "log_probs", "rewards",
          "episode_starts", "dones", "advantages", "returns")


@pytest.mark.parametrize("F,N,goal,T,mode,max_steps,det", [
    (300, 5, True, 10, "mt19937", 13, False),    # reset events inside rollouts, 12 fm / wave
    (1001, 10, True, 10, "philox", 23, False),   # BASELINE config-2 shape (scaled), tail wave
    (37, 64, True, 6, "mt19937", 9, False),      # one formation per wavefront
    (50, 7, False, 8, "philox", 11, True),       # D = 6, 9 formations / wave, deterministic
    (40, 5, True, 20, "philox", 7, False),       # T = 20: long rollout, several resets
    (9, 33, True, 3, "mt19937", 1000, False),    # M = 33: second tile has one agent
])
def test_fused_rollout_matches_unfused(mods, F, N, goal, T, mode, max_steps, det):
    """fenv_policy_rollout (one kernel per rollout) == policy_forward + fenv_step per step +
    rollout_gae, bit for bit, over several consecutive rollouts (episode boundaries inside)."""
    D = 8 if goal else 6
    cfg = {"num_formation": F, "num_agents_per_formation": N, "goal_in_obs": goal}
    ve, ro = mods["vectorized_env"], mods["rollout"]
    envs = [ve.FormationEnv(cfg, device=DEV, seed=4, reset_mode=mode, max_steps=max_steps)
            for _ in range(2)]
    pol = mods["policy"].MlpPolicy(D, device=DEV, seed=1)
    g = torch.Generator().manual_seed(N)
    with torch.no_grad():  # non-trivial heads so actions move the agents
        pol.flat.add_(torch.randn(pol.flat.shape, generator=g).to(DEV) * 0.05)
    bufs = [ro.RolloutBuffer(T, F * N, D, DEV) for _ in range(2)]
    cols = [ro.RolloutCollector(envs[0], pol, bufs[0], seed=7, fused=True),
            ro.RolloutCollector(envs[1], pol, bufs[1], seed=7, fused=False)]
    saw_done = False
    for r in range(4):
        for c in cols:
            c.collect(deterministic=det)
        torch.cuda.synchronize()
        for name in FIELDS:
            a, b = getattr(bufs[0], name), getattr(bufs[1], name)
            assert torch.equal(a, b), f"rollout {r}: {name} differs"
        saw_done |= bool(bufs[0].dones.any())
        assert torch.equal(cols[0].last_obs, cols[1].last_obs)
        assert torch.equal(cols[0].last_episode_starts, cols[1].last_episode_starts)
        assert torch.equal(cols[0]._last_values, cols[1]._last_values)
        for sa, sb in zip(envs[0].get_state(), envs[1].get_state()):
            assert torch.equal(sa, sb), f"rollout {r}: env state differs"
    assert cols[0].num_timesteps == cols[1].num_timesteps == 4 * T * F * N
    if max_steps + 2 <= 4 * T:
        assert saw_done


def test_fused_rollout_errors(mods, flib):
    ve, ro = mods["vectorized_env"], mods["rollout"]
    env = ve.FormationEnv({"num_formation": 3, "num_agents_per_formation": 65,
                           "goal_in_obs": True}, device=DEV, seed=0)
    pol = mods["policy"].MlpPolicy(8, device=DEV)
    col = ro.RolloutCollector(env, pol, ro.RolloutBuffer(4, 195, 8, DEV), seed=0)
    assert not col.fused  # N > 64 falls back to the per-step HIP path
    col.collect()
    with pytest.raises(flib.FenvError, match="num_agents must be <= 64"):
        ro.RolloutCollector(env, pol, ro.RolloutBuffer(4, 195, 8, DEV), fused=True).collect()
    env2 = ve.FormationEnv({"num_formation": 3, "num_agents_per_formation": 5,
                            "goal_in_obs": True}, device=DEV, seed=0, max_steps=3)
    with pytest.raises(flib.FenvError, match="more than one reset event"):
        ro.RolloutCollector(env2, pol, ro.RolloutBuffer(12, 15, 8, DEV), fused=True).collect()


def test_graph_update_matches_eager(mods):
    """The HIP-graph minibatch update (one replay per minibatch) == the eager loop: same
    minibatches (same randperm per epoch), same parameters after train(), same loss stats."""
    cfg = {"num_formation": 64, "num_agents_per_formation": 5, "goal_in_obs": True}
    runs = []
    for graph in (False, True):
        env = mods["vectorized_env"].FormationEnv(cfg, device=DEV, seed=1, reset_mode="philox")
        # 3,200 samples / 256 = 12 full minibatches + a partial one of 128
        ppo = mods["ppo"].PPO(env, mods["ppo"].PPOConfig(batch_size=256, n_epochs=3), seed=4,
                              use_graph=graph)
        for _ in range(2):  # the second train() replays the graphs captured by the first
            with torch.no_grad():
                ppo.collector.collect()
            st = ppo.train()
        runs.append((ppo.policy.flat.clone(), st))
    (p0, s0), (p1, s1) = runs
    torch.testing.assert_close(p1, p0, atol=1e-6, rtol=1e-5)
    for k in s0:
        assert abs(s0[k] - s1[k]) <= 1e-5 * max(1.0, abs(s0[k])), k


@pytest.mark.parametrize("goal", [True, False])
def test_fused_update_matches_torch(mods, goal):
    """ppo_update (one HIP kernel for all epochs x minibatches: loss, backward, grad clip,
    Adam) == the torch autograd update on the same samples and permutations, to fp32
    summation-order rounding: 2 epochs x 13 minibatches of 64 (the last one 32)."""
    cfg = {"num_formation": 16, "num_agents_per_formation": 5, "goal_in_obs": goal}
    runs = []
    for fused in (False, True):
        env = mods["vectorized_env"].FormationEnv(cfg, device=DEV, seed=1, reset_mode="philox")
        ppo = mods["ppo"].PPO(env, mods["ppo"].PPOConfig(batch_size=64, n_epochs=2), seed=4,
                              use_graph=False, use_fused=fused)
        flat0 = ppo.policy.flat.clone()
        for _ in range(2):
            with torch.no_grad():
                ppo.collector.collect()
            st = ppo.train()
        s = ppo.opt.state[ppo.param]
        runs.append((flat0, ppo.policy.flat.clone(), st, s["exp_avg"].clone(),
                     s["exp_avg_sq"].clone(), float(s["step"])))
    (a0, p0, s0, m0, v0, k0), (a1, p1, s1, m1, v1, k1) = runs
    assert torch.equal(a0, a1)
    assert k0 == k1 == 2 * 2 * 13
    moved = (p0 - a0).abs().max().item()
    err = (p1 - p0).abs().max().item()
    assert moved > 1e-3 and err < 1e-3 * moved, (moved, err)
    torch.testing.assert_close(m1, m0, atol=1e-6, rtol=1e-3)
    torch.testing.assert_close(v1, v0, atol=1e-9, rtol=1e-3)
    for k in s0:
        assert abs(s0[k] - s1[k]) <= 1e-4 * max(1.0, abs(s0[k])), (k, s0[k], s1[k])


def test_fused_update_repeatable(mods):
    """The two-CU fused update (actor and critic blocks exchanging the gradient norm through L2
    every minibatch) is deterministic: 8 launches from the same parameters / Adam state / samples
    at the reference's training config (1000 x 5 agents, 10 epochs x 782 minibatches) give
    bit-identical parameters, Adam moments and loss sums, with no launch re-run after a lost
    exchange (ppo.py exchange_retries, profiles/ab/r2_ppo_exchange_ab.txt)."""
    cfg = {"num_formation": 1000, "num_agents_per_formation": 5, "goal_in_obs": True}
    env = mods["vectorized_env"].FormationEnv(cfg, device=DEV, seed=2, reset_mode="philox")
    ppo = mods["ppo"].PPO(env, mods["ppo"].PPOConfig(), seed=3, use_graph=False, use_fused=True)
    with torch.no_grad():
        ppo.collector.collect()
    ppo.train()  # creates the Adam state
    with torch.no_grad():
        ppo.collector.collect()
    st = ppo.opt.state[ppo.param]
    state = (ppo.param, st["exp_avg"], st["exp_avg_sq"], st["step"])
    snap = tuple(t.detach().clone() for t in state)
    gen = ppo.gen.get_state()  # the epochs' permutations are drawn from it
    ref = None
    for r in range(8):
        with torch.no_grad():
            for t, s in zip(state, snap):
                t.copy_(s)
        ppo.gen.set_state(gen)
        stats = ppo.train()
        out = tuple(t.detach().clone() for t in state) + (stats,)
        if ref is None:
            ref = out
            continue
        for k in range(4):
            assert torch.equal(out[k], ref[k]), (r, k)
        assert out[4] == ref[4], r
    assert ppo.exchange_retries == 0


@pytest.mark.parametrize("mode", ["mt19937", "philox"])
def test_sharded_rollouts_concatenate_to_unsharded(mods, mode):
    """Shards of one batch (uneven: 26 + 25 formations) collect, between them, exactly the
    unsharded rollout: env shards are bit-exact (MT19937 skip-ahead / Philox by global
    formation) and the policy noise is keyed by global agent index (fenv_policy_rollout,
    policy_forward row0).  Fused and per-step paths alike, several rollouts with resets."""
    ve, ro = mods["vectorized_env"], mods["rollout"]
    F, N, T = 51, 5, 10
    pol = mods["policy"].MlpPolicy(8, device=DEV, seed=6)
    with torch.no_grad():
        pol.flat.add_(torch.randn(pol.flat.shape, generator=torch.Generator().manual_seed(1))
                      .to(DEV) * 0.05)
    cfg = lambda f: {"num_formation": f, "num_agents_per_formation": N, "goal_in_obs": True}  # noqa
    for fused in (True, False):
        whole = ve.FormationEnv(cfg(F), device=DEV, seed=9, reset_mode=mode, max_steps=12)
        parts = [ve.FormationEnv(cfg(c), device=DEV, seed=9, reset_mode=mode, max_steps=12,
                                 first_formation=f0, total_formations=F)
                 for f0, c in ((0, 26), (26, 25))]
        bufs = [ro.RolloutBuffer(T, e.num_envs, 8, DEV) for e in [whole] + parts]
        cols = [ro.RolloutCollector(e, pol, b, seed=21, fused=fused)
                for e, b in zip([whole] + parts, bufs)]
        for r in range(3):
            for c in cols:
                c.collect()
            torch.cuda.synchronize()
            for name in FIELDS:
                cat = torch.cat([getattr(bufs[1], name), getattr(bufs[2], name)], dim=1)
                assert torch.equal(getattr(bufs[0], name), cat), (fused, r, name)
        assert bool(bufs[0].dones.any()) or bool(torch.cat([b.dones for b in bufs]).any())


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ppo_rank(rank, world, port, q, F, kw):
    """One rank of a world-2 PPO run on cuda:0 (gloo: both ranks share the one GPU)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    import pkgload
    pkg = pkgload.load()
    from importlib import import_module
    d = import_module(pkg.__name__ + ".distributed")
    ve = import_module(pkg.__name__ + ".vectorized_env")
    ppo_mod = import_module(pkg.__name__ + ".ppo")
    d.init_from_env(backend="gloo")
    first, count = d.shard_range(F, rank, world)
    env = ve.FormationEnv({"num_formation": count, "num_agents_per_formation": 5,
                           "goal_in_obs": True}, device=DEV, seed=2, first_formation=first,
                          total_formations=F, **kw["env"])
    m = ppo_mod.PPO(env, ppo_mod.PPOConfig(**kw["ppo"]), seed=3)
    m.learn(total_timesteps=kw["timesteps"])
    st = m.opt.state[m.param]
    q.put((rank, m.policy.flat.cpu().numpy().tobytes(), st["exp_avg"].cpu().numpy().tobytes(),
           float(st["step"]), m.num_timesteps, m._gsamples.cpu().numpy().tobytes()))
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("batch_size,n_epochs", [(64, 2), (512, 2)])  # fused kernel / graphs
def test_two_rank_ppo_equals_single_process(mods, batch_size, n_epochs):
    """World-2 training (uneven shards 26 + 25 formations, gloo, both ranks on this GPU): one
    all-gather of the samples per update, the same update on every rank -- both ranks end with
    bitwise identical parameters and Adam state, equal to a single-process run on the unsharded
    env (which also equals train() on the concatenated shard buffers), and agree on
    num_timesteps.  No per-minibatch collective exists to hang on uneven shards."""
    F = 51
    kw = {"env": {"reset_mode": "mt19937", "max_steps": 12},
          "ppo": {"batch_size": batch_size, "n_epochs": n_epochs}, "timesteps": F * 5 * 10 * 3}
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ppo_rank, args=(r, 2, port, q, F, kw)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r[0], r[1:]) for r in (q.get(timeout=300), q.get(timeout=300)))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    # single process, unsharded
    env = mods["vectorized_env"].FormationEnv({"num_formation": F, "num_agents_per_formation": 5,
                                               "goal_in_obs": True}, device=DEV, seed=2,
                                              **kw["env"])
    m = mods["ppo"].PPO(env, mods["ppo"].PPOConfig(**kw["ppo"]), seed=3)
    m.learn(total_timesteps=kw["timesteps"])
    st = m.opt.state[m.param]
    assert m.num_timesteps == res[0][3] == res[1][3] == kw["timesteps"]
    assert res[0][0] == res[1][0], "ranks' parameters differ"
    assert res[0][1] == res[1][1] and res[0][2] == res[1][2], "ranks' Adam states differ"
    assert res[0][4] == res[1][4], "ranks gathered different samples"
    b = m.buffer
    D = 8
    g = np.frombuffer(res[0][4], np.float32).reshape(10, F * 5, D + 5)
    assert np.array_equal(g[..., :D], b.observations.cpu().numpy())
    assert np.array_equal(g[..., D + 3], b.advantages.cpu().numpy())
    assert res[0][0] == m.policy.flat.cpu().numpy().tobytes(), "world-2 != single process"
    assert res[0][1] == st["exp_avg"].cpu().numpy().tobytes()
