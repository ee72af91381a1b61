"""GPU: device rollout collection, GAE kernel and the on-device PPO update.

GAE is checked against a numpy restatement of SB3 RolloutBuffer.compute_returns_and_advantage
(parity unpinned vs SB3 itself, which is not installed); the rollout against step-by-step
policy + env calls; the training-side torch model against the HIP policy kernel."""
import numpy as np
import pytest
import torch

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


def test_collect_matches_stepwise(mods):
    F, N = 300, 5
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
    torch.testing.assert_close(v, r["value"], atol=2e-5, rtol=2e-5)
    torch.testing.assert_close(lp, r["log_prob"], atol=1e-4, rtol=1e-5)
    assert torch.allclose(ent, torch.full_like(ent, 2 * (0.5 + 0.5 * np.log(2 * np.pi))))


def test_ppo_learns(mods):
    cfg = {"num_formation": 256, "num_agents_per_formation": 5, "goal_in_obs": True}
    env = mods["vectorized_env"].FormationEnv(cfg, device=DEV, seed=0, reset_mode="philox")
    ppo = mods["ppo"].PPO(env, mods["ppo"].PPOConfig(batch_size=1024, n_epochs=4), seed=0)
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
