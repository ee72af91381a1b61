"""GPU: training entry point, SB3-layout checkpoints and policy playback:
the reference's ``python vectorized_env.py name=...`` (vectorized_env.py:112-137) and
``python visualize_policy.py name=...`` (visualize_policy.py:23-48) on the HIP path."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def mods(pkg):
    from importlib import import_module
    return {m: import_module(pkg.__name__ + "." + m)
            for m in ("ppo", "policy", "vectorized_env", "checkpoint", "train",
                      "visualize_policy")}


def test_ppo_checkpoints_and_reload(mods, tmp_path):
    cfg = {"num_formation": 16, "num_agents_per_formation": 5, "goal_in_obs": True}
    env = mods["vectorized_env"].FormationEnv(cfg, device=DEV, seed=0, reset_mode="philox")
    ppo = mods["ppo"].PPO(env, mods["ppo"].PPOConfig(batch_size=256, n_epochs=2), seed=0)
    cb = mods["checkpoint"].CheckpointCallback(10, str(tmp_path))
    A = env.num_envs
    ppo.learn(total_timesteps=3 * 10 * A, callback=cb)
    names = sorted(os.listdir(tmp_path), key=lambda n: int(n.split("_")[-2]))
    assert names == [f"rl_model_{k * 10 * A}_steps.zip" for k in (1, 2, 3)]
    # save -> load: identical policy bits and identical kernel outputs
    p = ppo.save(str(tmp_path / "final"))
    pol = mods["policy"].MlpPolicy.from_checkpoint(p, device=DEV)
    assert torch.equal(pol.flat, ppo.policy.flat)
    obs = torch.rand((1000, 8), device=DEV) * 2 - 1
    a = ppo.policy.forward(obs, deterministic=True)
    b = pol.forward(obs, deterministic=True)
    assert torch.equal(a["mu"], b["mu"]) and torch.equal(a["value"], b["value"])
    ppo2 = mods["ppo"].PPO.load(p, env)
    assert torch.equal(ppo2.policy.flat, ppo.policy.flat)
    assert ppo2.cfg.batch_size == 256 and ppo2.loaded_num_timesteps == ppo.num_timesteps


def test_train_entry_point_and_playback(mods, tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    out = mods["train"].main(["name=t1", "num_formation=8", "num_agents_per_formation=5",
                              "num_steps=30", "batch_size=256", "n_epochs=1", "seed=3"])
    assert out == os.path.join(str(tmp_path), "logs", "t1")
    # total_timesteps = 30 * 8 = 240 < one rollout (10 steps x 40 agents): one checkpoint
    assert os.listdir(out) == ["rl_model_400_steps.zip"]
    cfgm = mods["visualize_policy"]._pkg()
    from importlib import import_module
    config = import_module(cfgm.__name__ + ".config")
    cfg = config.load_config(overrides=["name=t1"])
    path = mods["checkpoint"].latest_checkpoint(out)
    pb = mods["visualize_policy"].Playback(cfg, path, device=DEV, visualize=True, verbose=False)
    assert pb.env.num_envs == 5 and pb.first_env.fig is not None
    o0 = pb.obs.copy()
    for i in range(3):
        rew, done = pb.simulate_func(i)
        assert rew.shape == (5,) and done.shape == (5,)
    assert not np.array_equal(o0, pb.obs)
    # the actions it took are the deterministic policy's clipped means
    act, _ = pb.model.predict(pb.obs, deterministic=True)
    assert np.all(np.abs(act) <= 1)


def test_visualize_main_saves_animation(mods, tmp_path, monkeypatch):
    pytest.importorskip("PIL")
    monkeypatch.chdir(tmp_path)
    mods["train"].main(["name=t2", "num_formation=4", "num_steps=10", "batch_size=128",
                        "n_epochs=1"])
    gif = tmp_path / "play.gif"
    mods["visualize_policy"].main(["name=t2", "steps_to_simulate=3", f"save={gif}", "quiet=true"])
    assert gif.exists() and gif.stat().st_size > 0
