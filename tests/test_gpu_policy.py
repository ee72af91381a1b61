"""GPU parity of the policy forward (policy_forward, split-f16 MFMA kernel) against the torch-CPU
fp32 restatement of SB3's ActorCriticPolicy (oracle/policy_oracle.py; parity unpinned vs SB3
itself, which is not installed).

Tolerance: the north star's 1e-5 relative (tests/tolerance.py): |err| <= 1e-5 * (|ref| + s),
s = RMS of the output over the batch -- mu, value, the sampled action and log_prob alike (the
kernel differs from torch in summation order, its tanh and its Box-Muller transcendentals)."""
import numpy as np
import pytest
import torch

import policy_oracle as po
from tolerance import assert_rel_close

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def pol_mod(pkg):
    from importlib import import_module
    return import_module(pkg.__name__ + ".policy")


def randomize(pol, seed):
    g = torch.Generator().manual_seed(seed)
    sd = pol.state_dict()
    for k, v in sd.items():
        if k.endswith("bias"):
            sd[k] = torch.randn(v.shape, generator=g) * 0.3
        elif k == "log_std":
            sd[k] = torch.randn(v.shape, generator=g) * 0.5
        else:
            sd[k] = v + torch.randn(v.shape, generator=g) * 0.05
    pol.load_state_dict(sd)
    return sd


@pytest.mark.parametrize("D", [8, 6])
@pytest.mark.parametrize("B", [1, 31, 32, 33, 1000, 65543])
def test_deterministic_forward(pol_mod, D, B):
    pol = pol_mod.MlpPolicy(D, device=DEV, seed=B)
    sd = randomize(pol, B + D)
    g = torch.Generator().manual_seed(B)
    obs = (torch.rand((B, D), generator=g) * 2.4 - 1.2)
    r = pol.forward(obs.to(DEV), deterministic=True)
    mu, val = po.forward(sd, obs)
    assert_rel_close(r["mu"], mu, "mu")
    assert_rel_close(r["value"], val, "value")
    assert_rel_close(r["action"], mu, "action")
    assert_rel_close(r["clipped"], mu.clamp(-1, 1), "clipped")
    assert_rel_close(r["log_prob"], po.log_prob(sd, mu, mu), "log_prob")


def test_large_preactivations(pol_mod):
    """Saturating tanh inputs (|x| >> 1) and tiny ones (|x| < 0.3, the polynomial branch)."""
    pol = pol_mod.MlpPolicy(8, device=DEV, seed=1)
    sd = randomize(pol, 9)
    for scale in (1e-4, 0.05, 3.0, 40.0):
        obs = (torch.rand((4096, 8), generator=torch.Generator().manual_seed(2)) * 2 - 1) * scale
        r = pol.forward(obs.to(DEV), deterministic=True)
        mu, val = po.forward(sd, obs)
        assert_rel_close(r["mu"], mu, f"mu scale {scale}")
        assert_rel_close(r["value"], val, f"value scale {scale}")


def test_stochastic_sample_and_log_prob(pol_mod):
    B, seed, off = 50000, 77, 5
    pol = pol_mod.MlpPolicy(8, device=DEV, seed=4)
    sd = randomize(pol, 4)
    obs = torch.rand((B, 8), generator=torch.Generator().manual_seed(3)) * 2 - 1
    r = pol.forward(obs.to(DEV), deterministic=False, seed=seed, offset=off)
    mu, _ = po.forward(sd, obs)
    eps = torch.from_numpy(po.philox_normals(B, seed, off)).float()
    std = sd["log_std"].exp()
    a = mu.double() + std.double() * torch.from_numpy(po.philox_normals(B, seed, off))
    assert_rel_close(r["action"], a, "action")
    act = r["action"].cpu()
    # log_prob of the kernel's own action under the oracle's mu (float64 Normal.log_prob)
    assert_rel_close(r["log_prob"], po.log_prob({"log_std": sd["log_std"].double()},
                                                mu.double(), act.double()), "log_prob")
    torch.testing.assert_close(r["clipped"].cpu(), act.clamp(-1, 1), atol=0, rtol=0)
    # the noise is standard normal
    e = ((act - r["mu"].cpu()) / std).numpy()
    assert abs(e.mean()) < 0.02 and abs(e.std() - 1) < 0.02
    # offset advances the stream; same (seed, offset) reproduces it
    r2 = pol.forward(obs.to(DEV), deterministic=False, seed=seed, offset=off)
    assert torch.equal(r2["action"], r["action"])
    r3 = pol.forward(obs.to(DEV), deterministic=False, seed=seed, offset=off + 1)
    assert not torch.equal(r3["action"], r["action"])
    # row0 keys the noise by global row: a shard's rows draw what the full batch draws
    R = 12345
    r4 = pol.forward(obs[R:].to(DEV), deterministic=False, seed=seed, offset=off, row0=R)
    assert torch.equal(r4["action"], r["action"][R:])
    assert torch.equal(r4["log_prob"], r["log_prob"][R:])


def test_state_dict_names_roundtrip(pol_mod):
    pol = pol_mod.MlpPolicy(8, device=DEV)
    sd = pol.state_dict()
    assert list(sd) == [k for k, _ in po.SB3_KEYS]
    assert sum(v.numel() for v in sd.values()) == 9669
    sd2 = {k: v + 1 for k, v in sd.items()}
    pol.load_state_dict(sd2)
    for k, v in pol.state_dict().items():
        assert torch.equal(v, sd2[k])
    with pytest.raises(KeyError):
        pol.load_state_dict({})


def test_policy_on_env_observations(pol_mod, venv):
    env = venv.FormationEnv({"num_formation": 512, "num_agents_per_formation": 10,
                             "goal_in_obs": True}, device=DEV, seed=2)
    obs = env.reset_tensor()
    pol = pol_mod.MlpPolicy(8, device=DEV, seed=0)
    r = pol.forward(obs, deterministic=True)
    mu, val = po.forward(pol.state_dict(), obs.cpu())
    assert_rel_close(r["mu"], mu, "mu")
    assert_rel_close(r["value"], val, "value")
    acts, _ = pol.predict(obs.cpu().numpy())
    assert acts.shape == (5120, 2) and np.all(np.abs(acts) <= 1)


def test_batch_beyond_int32_offsets_sampled(pol_mod):
    """Maximum sizes: 3e8 agents (obs element offsets pass 2^31; ~20 GB of HBM).  Rows are
    independent, so sampled rows -- incl. those around the 2^31-element boundary and the last,
    partial tile -- are checked against the oracle."""
    B, D = 300_000_001, 8
    pol = pol_mod.MlpPolicy(D, device=DEV, seed=3)
    sd = randomize(pol, 17)
    g = torch.Generator(device=DEV).manual_seed(4)
    obs = torch.rand((B, D), device=DEV, generator=g) * 2.4 - 1.2
    r = pol.forward(obs, deterministic=True)
    torch.cuda.synchronize()
    edge = (1 << 31) // D
    rows = np.unique(np.concatenate([np.random.default_rng(5).choice(B, 4000, replace=False),
                                     np.arange(edge - 40, edge + 40), np.arange(B - 70, B),
                                     [0, 1]]))
    idx = torch.from_numpy(rows).to(DEV)
    mu, val = po.forward(sd, obs[idx].cpu())
    assert_rel_close(r["mu"][idx], mu, "mu")
    assert_rel_close(r["value"][idx], val, "value")
    assert_rel_close(r["clipped"][idx], mu.clamp(-1, 1), "clipped")


def test_predict_zero_copy_matches_forward(pkg, pol_mod):
    """SB3 ``predict`` (visualize_policy.py:16) runs the kernel on device-mapped host memory: an
    env's numpy-face observations are read in place, other numpy arrays (plain, strided, sliced
    to an unaligned start) are copied into the policy's block first, and CUDA tensors go through
    ``forward``.  Every form returns the bits of ``forward(...)["clipped"]`` at the same noise
    offset -- deterministic and sampled -- as a fresh array that later calls leave alone."""
    from importlib import import_module
    venv = import_module(pkg.__name__ + ".vectorized_env")
    flib = import_module(pkg.__name__ + "._lib")
    env = venv.FormationEnv({"num_formation": 40, "num_agents_per_formation": 5,
                             "goal_in_obs": True}, log=False, device=DEV, seed=2,
                            reset_mode="philox")
    pol = pol_mod.MlpPolicy(8, device=DEV, seed=9)
    randomize(pol, 4)
    obs = env.reset()
    assert flib.device_address(obs) is not None          # lives in the env's host block
    assert flib.device_address(obs.copy()) is None
    assert flib.device_address(obs[1:]) is not None      # 32-B rows keep 16-B alignment
    raw = np.zeros(obs.size + 1, np.float32)
    unaligned = raw[1:].reshape(obs.shape)               # 4-B aligned start: copied first
    unaligned[...] = obs
    forms = {"env": obs, "env_rows": obs[40:], "plain": obs.copy(),
             "strided": np.asfortranarray(obs), "unaligned": unaligned}
    kept = []
    for det in (True, False):
        for name, o in forms.items():
            off = pol._offset
            ref = pol.forward(torch.from_numpy(np.ascontiguousarray(o)).to(DEV),
                              deterministic=det, offset=off)["clipped"].cpu().numpy()
            pol._offset = off
            got, st = pol.predict(o, deterministic=det)
            assert st is None and got.shape == (o.shape[0], 2)
            assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), (name, det)
            assert pol._offset == off + 1
            kept.append((got, got.copy()))
    t = torch.from_numpy(obs.copy()).to(DEV)
    off = pol._offset
    ref = pol.forward(t, deterministic=True, offset=off)["clipped"].cpu().numpy()
    pol._offset = off
    assert np.array_equal(pol.predict(t)[0], ref)
    # a different batch size replaces the cached block; earlier results are untouched
    o2, _, _, _ = env.step(np.zeros((200, 2), np.float32))
    assert pol.predict(o2[:40])[0].shape == (40, 2)
    for got, snap in kept:
        assert np.array_equal(got, snap)
    with pytest.raises(ValueError):
        pol.predict(np.zeros((4, 6), np.float32))
    # an empty batch advances the noise offset exactly as forward() does
    off = pol._offset
    got, _ = pol.predict(np.zeros((0, 8), np.float32))
    assert got.shape == (0, 2) and pol._offset == off + 1
    pol.forward(torch.zeros((0, 8), device=DEV))
    assert pol._offset == off + 2
    env.release()
