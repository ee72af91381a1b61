"""CPU: SB3-layout checkpoint zips, the CheckpointCallback schedule and the newest-checkpoint
rule of the reference (vectorized_env.py:124, visualize_policy.py:29-35).  Parity against SB3
itself is unpinned (SB3 is not installed); the layout follows SB3 2.x save_to_zip_file."""
import io
import json
import os
import zipfile

import pytest
import torch


@pytest.fixture(scope="module")
def ck(pkg):
    from importlib import import_module
    return import_module(pkg.__name__ + ".checkpoint")


@pytest.fixture(scope="module")
def shapes(pkg):
    from importlib import import_module
    pol = import_module(pkg.__name__ + ".policy")
    return [(k, pol._shape(s, 8)) for k, s in pol.PARAM_SPECS]


def random_sd(shapes, seed=0):
    g = torch.Generator().manual_seed(seed)
    return {k: torch.randn(s, generator=g) for k, s in shapes}


def test_zip_roundtrip_and_layout(ck, shapes, tmp_path):
    sd = random_sd(shapes)
    p = ck.save_sb3_zip(str(tmp_path / "m"), sd, num_timesteps=1234, data={"n_steps": 10})
    assert p.endswith("m.zip") and os.path.exists(p)
    with zipfile.ZipFile(p) as z:
        names = set(z.namelist())
        assert {"data", "policy.pth", "pytorch_variables.pth", "_stable_baselines3_version",
                "system_info.txt"} <= names
        data = json.loads(z.read("data"))
        # policy.pth is a plain tensor dict: the safe loader reads it
        sd2 = torch.load(io.BytesIO(z.read("policy.pth")), weights_only=True)
    assert data["num_timesteps"] == 1234 and data["n_steps"] == 10
    assert {"policy_class", "observation_space", "action_space"} <= set(data)
    assert list(sd2) == list(sd)
    sd3, data3 = ck.load_sb3_zip(p)
    assert data3 == data
    for k in sd:
        assert torch.equal(sd3[k], sd[k])


def _standin_modules(monkeypatch):
    """Stand-ins for the two classes the pickled entries name, restating what unpickling uses
    of them: gymnasium's Space.__setstate__ / Box.__setstate__ (legacy-key handling, then a
    __dict__ update; low_repr / high_repr re-derived when absent) and SB3's policy class."""
    import sys
    import types

    class Box:
        @property
        def shape(self):
            return self._shape

        def __setstate__(self, state):
            state = dict(state)
            if "shape" in state:
                state["_shape"] = state.pop("shape")
            if "np_random" in state:
                state["_np_random"] = state.pop("np_random")
            self.__dict__.update(state)

    class ActorCriticPolicy:
        pass

    mods = {}
    for name in ("gymnasium", "gymnasium.spaces", "gymnasium.spaces.box", "stable_baselines3",
                 "stable_baselines3.common", "stable_baselines3.common.policies"):
        mods[name] = types.ModuleType(name)
        monkeypatch.setitem(sys.modules, name, mods[name])
    Box.__module__, ActorCriticPolicy.__module__ = "gymnasium.spaces.box", \
        "stable_baselines3.common.policies"
    mods["gymnasium.spaces.box"].Box = Box
    mods["stable_baselines3.common.policies"].ActorCriticPolicy = ActorCriticPolicy
    return Box, ActorCriticPolicy


def test_pickled_entries_load_as_sb3_does(ck, shapes, tmp_path, monkeypatch):
    """What SB3's PPO.load (save_util.json_to_data: base64 -> cloudpickle.loads) gets from the
    three pickled ``data`` entries, which the reference's playback needs with no custom_objects
    (visualize_policy.py:35): the policy class and the reference's two Box spaces
    (vectorized_env.py:34-35).  Parity against SB3 / gymnasium themselves: unpinned."""
    import base64
    import pickle
    import warnings

    import numpy as np
    Box, ACP = _standin_modules(monkeypatch)
    p = ck.save_sb3_zip(str(tmp_path / "m"), random_sd(shapes), num_timesteps=7)
    with zipfile.ZipFile(p) as z:
        data = json.loads(z.read("data"))
    assert data["policy_class"][":type:"] == "<class 'abc.ABCMeta'>"
    assert data["observation_space"][":type:"] == "<class 'gymnasium.spaces.box.Box'>"
    assert data["policy_kwargs"] == {}
    out = {}
    with warnings.catch_warnings():
        warnings.simplefilter("error")  # numpy.core names must load without a deprecation
        for k in ("policy_class", "observation_space", "action_space"):
            out[k] = pickle.loads(base64.b64decode(data[k][":serialized:"].encode()))
    assert out["policy_class"] is ACP
    for k, dim in (("observation_space", 8), ("action_space", 2)):
        b = out[k]
        assert type(b) is Box and b.shape == (dim,) and b.dtype == np.float32
        assert b.low.dtype == np.float32 and b.high.dtype == np.float32
        assert np.array_equal(b.low, np.full(dim, -1, np.float32))
        assert np.array_equal(b.high, np.full(dim, 1, np.float32))
        assert b.bounded_below.dtype == np.bool_ and b.bounded_below.all()
        assert b.bounded_above.all() and b.low_repr == "-1.0" and b.high_repr == "1.0"
        assert b._np_random is None and b.low.flags.writeable


def test_optimizer_group_is_sb3s(ck, shapes):
    """The saved Adam param group carries SB3's optimizer settings (a non-capturable Adam), so
    SB3's set_parameters loads it on any device; lr / betas / eps are the trained ones."""
    n = sum(int(torch.tensor(s).prod()) for _, s in shapes)
    p = torch.nn.Parameter(torch.zeros(n))
    opt = torch.optim.Adam([p], lr=1e-3, eps=1e-5, capturable=False)
    p.grad = torch.ones(n)
    opt.step()
    sd = opt.state_dict()
    sd["param_groups"][0]["capturable"] = True
    g = ck.optimizer_state_from_flat(shapes, sd)["param_groups"][0]
    assert g["capturable"] is False and g["foreach"] is None and g["fused"] is None
    assert g["lr"] == 1e-3 and g["eps"] == 1e-5 and tuple(g["betas"]) == (0.9, 0.999)
    assert g["params"] == list(range(13))


def test_zip_rejects_incomplete_state(ck, shapes, tmp_path):
    sd = random_sd(shapes)
    del sd["log_std"]
    with pytest.raises(KeyError):
        ck.save_sb3_zip(str(tmp_path / "bad.zip"), sd, num_timesteps=1)
    with zipfile.ZipFile(tmp_path / "notmodel.zip", "w") as z:
        z.writestr("data", "{}")
    with pytest.raises(ValueError):
        ck.load_sb3_zip(str(tmp_path / "notmodel.zip"))


def test_optimizer_state_sliced_per_sb3_tensor(ck, shapes):
    n = sum(torch.Size(s).numel() for _, s in shapes)
    flat = torch.nn.Parameter(torch.zeros(n))
    opt = torch.optim.Adam([flat], lr=1e-3, eps=1e-5)
    flat.grad = torch.arange(n, dtype=torch.float32)
    opt.step()
    st = ck.optimizer_state_from_flat(shapes, opt.state_dict())
    assert st["param_groups"][0]["params"] == list(range(13))
    assert st["param_groups"][0]["eps"] == 1e-5
    offs, o = {}, 0
    for k, s in shapes:
        offs[k] = o
        o += torch.Size(s).numel()
    for i, k in enumerate(ck.SB3_PARAM_ORDER):
        s = dict(shapes)[k]
        ea = st["state"][i]["exp_avg"]
        assert tuple(ea.shape) == tuple(s)
        exp = opt.state_dict()["state"][0]["exp_avg"][offs[k]:offs[k] + ea.numel()].reshape(s)
        assert torch.equal(ea, exp)


def test_optimizer_state_roundtrip_to_flat(ck, shapes):
    """SB3's per-tensor Adam state (as policy.optimizer.pth holds it) back onto the flat
    parameter: the exact moments and step that were saved (PPO.load restores them)."""
    n = sum(torch.Size(s).numel() for _, s in shapes)
    flat = torch.nn.Parameter(torch.zeros(n))
    opt = torch.optim.Adam([flat], lr=1e-3, eps=1e-5)
    for k in range(3):
        flat.grad = torch.randn(n, generator=torch.Generator().manual_seed(k))
        opt.step()
    sb3 = ck.optimizer_state_from_flat(shapes, opt.state_dict())
    buf = io.BytesIO()
    torch.save(sb3, buf)  # what save_sb3_zip writes; read back with the safe loader
    sb3 = torch.load(io.BytesIO(buf.getvalue()), weights_only=True)
    back = ck.optimizer_state_to_flat(shapes, sb3, "cpu")
    st = opt.state_dict()["state"][0]
    assert torch.equal(back["exp_avg"], st["exp_avg"])
    assert torch.equal(back["exp_avg_sq"], st["exp_avg_sq"])
    assert float(back["step"]) == 3.0
    assert ck.optimizer_state_to_flat(shapes, None, "cpu") is None
    assert ck.optimizer_state_to_flat(shapes, {"state": {}, "param_groups": []}, "cpu") is None
    bad = {"state": {0: {"exp_avg": torch.zeros(3), "exp_avg_sq": torch.zeros(3), "step": 1}}}
    assert ck.optimizer_state_to_flat(shapes, bad, "cpu") is None


def test_sb3_pickled_hyperparameters_skipped(ck, pkg):
    """SB3 stores clip_range / learning_rate as cloudpickled schedules ({":type:", ":serialized:"}
    dicts in ``data``): PPO.load must not feed them to PPOConfig."""
    from importlib import import_module
    ppo = import_module(pkg.__name__ + ".ppo")
    data = {"clip_range": {":type:": "<class 'function'>", ":serialized:": "gAWV..."},
            "learning_rate": {":type:": "<class 'function'>", ":serialized:": "gAWV..."},
            "n_steps": 10, "batch_size": 64, "gamma": 0.99, "ent_coef": 0.01,
            "normalize_advantage": True, "n_epochs": "10", "vf_coef": True, "gae_lambda": 1}
    got = ck.plain_hyperparameters(data, ppo.PPOConfig)
    assert got == {"n_steps": 10, "batch_size": 64, "gamma": 0.99, "ent_coef": 0.01,
                   "normalize_advantage": True, "gae_lambda": 1.0}
    cfg = ppo.PPOConfig(**got)
    assert cfg.clip_range == 0.2 and cfg.learning_rate == 1e-3


def test_latest_checkpoint_rule(ck, shapes, tmp_path):
    for t in (20, 100, 3, 99):
        (tmp_path / ck.checkpoint_name(t)).write_bytes(b"")
    (tmp_path / "notes.txt").write_text("x")
    # a partial file a crashed save could leave behind is never picked
    (tmp_path / "rl_model_500_steps.zip.tmp").write_bytes(b"")
    assert ck.latest_checkpoint(str(tmp_path)).endswith("rl_model_100_steps.zip")
    # save_sb3_zip's own partial file does not look like a checkpoint
    ck.save_sb3_zip(str(tmp_path / ck.checkpoint_name(7)), random_sd(shapes), num_timesteps=7)
    assert not [f for f in os.listdir(tmp_path) if "partial" in f]
    assert ck.latest_checkpoint(str(tmp_path)).endswith("rl_model_100_steps.zip")
    (tmp_path / "empty").mkdir()
    with pytest.raises(FileNotFoundError):
        ck.latest_checkpoint(str(tmp_path / "empty"))


class FakeModel:
    def __init__(self):
        self.num_timesteps = 0
        self.saves = []

    def save(self, path, num_timesteps):
        self.saves.append((os.path.basename(path), num_timesteps))


@pytest.mark.parametrize("save_freq,n_steps", [(10, 10), (4, 10), (25, 10), (3, 1)])
def test_callback_schedule_matches_sb3(ck, save_freq, n_steps, tmp_path):
    """SB3: one _on_step per env step, save when n_calls % save_freq == 0, file named by the
    num_timesteps at that step."""
    A = 7
    m = FakeModel()
    cb = ck.CheckpointCallback(save_freq, str(tmp_path))
    expect = []
    calls = 0
    for rollout in range(6):
        for s in range(n_steps):
            calls += 1
            if calls % save_freq == 0:
                expect.append(ck.checkpoint_name((rollout * n_steps + s + 1) * A))
        m.num_timesteps += n_steps * A
        cb.on_steps(m, n_steps, A)
    assert [n for n, _ in m.saves] == expect
    assert all(t == int(n.split("_")[-2]) for n, t in m.saves)
    with pytest.raises(ValueError):
        ck.CheckpointCallback(0, str(tmp_path))


def test_train_cli_overrides(pkg):
    from importlib import import_module
    config = import_module(pkg.__name__ + ".config")
    cfg = config.load_config(overrides=["name=run7", "num_agents_per_formation=7",
                                        "+num_steps=30", "goal_in_obs=false"])
    assert (cfg.name, cfg.num_agents_per_formation, cfg.num_steps, cfg.goal_in_obs) == \
        ("run7", 7, 30, False)
