"""The C-ABI library (CPU-only checks: no kernel launches).

* libfenv.so loads and exports every function include/fenv.h declares;
* its host-side pieces (the reference's global MT19937 reset stream, desired neighbour
  distance) agree with the oracle;
* with no HIP device every env entry point fails loudly (no CPU fallback exists).
"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from oracle import COracleEnv, desired_neighbor_dist, mt_raw, torch_rand_from_raw

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_header_symbols_exported(flib):
    L = flib.lib()
    names = flib.header_symbols()
    assert "fenv_create" in names and "policy_forward" in names and "fenv_rollout" in names
    for n in names:
        assert hasattr(L, n), f"{n} declared in include/fenv.h but not exported"
    out = subprocess.run(["nm", "-D", "--defined-only", flib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    # the library carries gfx950 code objects only
    blob = open(flib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_signatures_cover_header(flib):
    assert set(flib.header_symbols()) <= set(flib.SIGNATURES)


@pytest.mark.parametrize("N", [1, 2, 3, 5, 7, 10, 64, 100, 1024, 1025, 5000, 1 << 24])
def test_desired_neighbor_dist(flib, N):
    assert np.float32(flib.lib().fenv_desired_neighbor_dist(N)) == desired_neighbor_dist(N)


@pytest.mark.parametrize("N,total,first,count,skip", [(5, 7, 0, 7, 0), (5, 7, 2, 3, 1),
                                                      (10, 4, 3, 1, 2), (64, 3, 1, 2, 0),
                                                      (1, 9, 4, 5, 3),
                                                      # discards of many whole 624-word blocks
                                                      # from every offset in a block
                                                      (5, 2000, 700, 300, 2), (7, 501, 13, 488, 5),
                                                      # >= 2^20 draws: drawn in 4 parts on 4
                                                      # threads (fenv_api.cpp draw_formations_par)
                                                      (5, 90000, 0, 90000, 1),
                                                      (10, 60001, 3001, 50003, 0)])
def test_host_reset_draws_match_torch_stream(flib, N, total, first, count, skip):
    """Draw set `skip` of the global stream, restricted to formations [first, first+count),
    equals torch.rand after torch.manual_seed (the reference's RNG, simulate.py:133-143)."""
    seed = 4242
    px = np.zeros(count * N, np.float32)
    py = np.zeros(count * N, np.float32)
    gx = np.zeros(count, np.float32)
    gy = np.zeros(count, np.float32)
    flib.check(flib.lib().fenv_host_reset_draws(seed, skip, total, first, count, N,
                                                *(flib.ptr(v) for v in (px, py, gx, gy))))
    per = 2 * N + 2
    g = torch.Generator().manual_seed(seed)
    allu = torch.rand(per * total * (skip + 1), generator=g).numpy()
    u = allu[per * total * skip:].reshape(total, per)[first:first + count]
    np.testing.assert_array_equal(px, (u[:, 0:2 * N:2] * np.float32(400)).reshape(-1))
    np.testing.assert_array_equal(py, (u[:, 1:2 * N:2] * np.float32(100)).reshape(-1))
    np.testing.assert_array_equal(gx, u[:, -2] * np.float32(280) + np.float32(60))
    np.testing.assert_array_equal(gy, u[:, -1] * np.float32(480) + np.float32(60))
    raw = mt_raw(seed, per * total * (skip + 1))
    assert np.array_equal(torch_rand_from_raw(raw), allu)


def test_host_reset_draws_equal_oracle_ctor_state(flib):
    F, N, seed = 6, 5, 77
    px = np.zeros(F * N, np.float32)
    py = np.zeros(F * N, np.float32)
    gx = np.zeros(F, np.float32)
    gy = np.zeros(F, np.float32)
    flib.check(flib.lib().fenv_host_reset_draws(seed, 0, F, 0, F, N,
                                                *(flib.ptr(v) for v in (px, py, gx, gy))))
    o = COracleEnv(F, N, True, seed).get_state()
    for a, b in zip((px, py, gx, gy), o[:4]):
        np.testing.assert_array_equal(a, b)


def test_bad_arguments_rejected_without_device(flib):
    L = flib.lib()
    assert L.fenv_host_reset_draws(1, 0, 2, 1, 5, 5, None, None, None, None) == -1
    assert b"bad arguments" in L.fenv_last_error()
    assert L.fenv_reduce_partials(None, 1, None, None) == -1
    assert L.policy_forward(None, 8, None, 1, 0, None, None, None, None, None, 0, 0, 0,
                            None) == -1
    assert L.policy_param_count(8) == 9669  # SURVEY §8(a) R10 (incl. log_std[2])


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-device failure path")
def test_create_fails_loudly_without_device(flib, venv):
    L = flib.lib()
    h = ctypes.c_void_p()
    rc = L.fenv_create(ctypes.byref(h), 0, 4, 5, 1, 0.25, 1000, 0, 0, 0, 4)
    assert rc != 0 and not h.value
    with pytest.raises(RuntimeError, match="no HIP device"):
        venv.FormationEnv({"num_formation": 2, "num_agents_per_formation": 5,
                           "goal_in_obs": True})


def test_invalid_config_rejected(flib):
    L = flib.lib()
    h = ctypes.c_void_p()
    assert L.fenv_create(ctypes.byref(h), 0, 4, 0, 1, 0.25, 1000, 0, 0, 0, 4) == -1
    assert L.fenv_create(ctypes.byref(h), 0, 4, 5, 1, 0.75, 1000, 0, 0, 0, 4) == -1
    assert L.fenv_create(ctypes.byref(h), 0, 4, 5, 1, 0.25, 1000, 0, 7, 0, 4) == -1
    assert L.fenv_create(ctypes.byref(h), 0, 4, 5, 1, 0.25, 1000, 0, 0, 2, 4) == -1


def test_ppo_update_validates_before_launch(flib):
    """ppo_update rejects bad arguments on the host (no kernel launch, no device needed)."""
    L = flib.lib()
    hp = flib.PPOHParams(clip_range=0.2, ent_coef=0.01, vf_coef=0.5, max_grad_norm=0.5, lr=1e-3,
                         beta1=0.9, beta2=0.999, eps=1e-5, normalize_advantage=1)
    fake = ctypes.c_void_p(0x1000)  # never dereferenced: validation fails first
    args = [fake] * 4 + [8] + [fake] * 5 + [100, fake, 1, 64, ctypes.byref(hp), fake, None]
    bad_bs = list(args)
    bad_bs[13] = 65
    assert L.ppo_update(*bad_bs) != 0
    assert b"batch_size" in L.fenv_last_error()
    bad_d = list(args)
    bad_d[4] = 7
    assert L.ppo_update(*bad_d) != 0
    nul = list(args)
    nul[0] = None
    assert L.ppo_update(*nul) != 0


SB3_STUB = r"""
import abc, sys, types
rec = {}
class VecEnv(abc.ABC):
    # SB3 2.x VecEnv: constructor arguments and abstract methods
    def __init__(self, num_envs, observation_space, action_space):
        rec.update(num_envs=num_envs, observation_space=observation_space,
                   action_space=action_space)
        self.num_envs = num_envs
        self.observation_space = observation_space
        self.action_space = action_space
        try:
            self.get_attr("render_modes")
        except AttributeError:
            rec["get_attr_raised"] = True
    for _m in ("reset", "step_async", "step_wait", "close", "get_attr", "set_attr",
               "env_method", "env_is_wrapped"):
        locals()[_m] = abc.abstractmethod(lambda self, *a, **k: None)
def mod(name, **kw):
    m = types.ModuleType(name); m.__dict__.update(kw); sys.modules[name] = m
mod("stable_baselines3"); mod("stable_baselines3.common")
mod("stable_baselines3.common.vec_env", VecEnv=VecEnv)
"""


def test_formation_env_is_sb3_vecenv_when_sb3_importable():
    """With an SB3 stand-in importable (the same sys.modules recipe gen_golden.py uses), the
    env subclasses SB3's VecEnv and calls its __init__ with the reference's arguments
    (vectorized_env.py:16, 36): num_envs = N * F and Box(-1, 1) spaces of shapes (D,) / (2,).
    Runs in a subprocess so the stand-in does not leak into other tests.  Without a device the
    constructor then fails loudly (no CPU path); GPU construction: tests/test_gpu_parity.py."""
    code = SB3_STUB + r"""
sys.path.insert(0, %r)
import pkgload
pkg = pkgload.load()
from importlib import import_module
ve = import_module(pkg.__name__ + ".vectorized_env")
assert issubclass(ve.FormationEnv, VecEnv), ve.FormationEnv.__mro__
assert not getattr(ve.FormationEnv, "__abstractmethods__", None)
env = ve.FormationEnv.__new__(ve.FormationEnv)
for m, args, exc in (("close", (), NotImplementedError), ("env_is_wrapped", (None,), NotImplementedError),
                     ("get_attr", ("x",), AttributeError), ("set_attr", ("x", 1), NotImplementedError),
                     ("env_method", ("x",), NotImplementedError), ("seed", (), NotImplementedError),
                     ("step_async", (None,), NotImplementedError), ("step_wait", (), NotImplementedError)):
    try:
        getattr(env, m)(*args)
    except exc:
        pass
    else:
        raise AssertionError(m)
try:
    ve.FormationEnv({"num_formation": 7, "num_agents_per_formation": 5, "goal_in_obs": False})
except RuntimeError as e:
    assert "no HIP device" in str(e) or "HIP" in str(e), e
import torch
if not torch.cuda.is_available():
    assert rec["num_envs"] == 35
    assert tuple(rec["observation_space"].shape) == (6,) and tuple(rec["action_space"].shape) == (2,)
    assert float(rec["action_space"].low.min()) == -1.0 and float(rec["action_space"].high.max()) == 1.0
    assert rec["get_attr_raised"]
print("ok")
""" % ROOT
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-3000:]


def test_formation_size_limits(pkg):
    """Any formation size the reference takes up to include/fenv.h's FENV_MAX_AGENTS (2^24) is
    accepted by the config layer (large formations run fenv_large.hip's kernels); 0 and larger
    sizes are rejected before anything is allocated."""
    from importlib import import_module
    cfgm = import_module(pkg.__name__ + ".config")
    for N in (1, 64, 1024, 1025, 5000, 1 << 24):
        cfgm.validate(cfgm.as_config({"num_formation": 2, "num_agents_per_formation": N}))
    for N in (0, (1 << 24) + 1):
        with pytest.raises(ValueError):
            cfgm.validate(cfgm.as_config({"num_formation": 2, "num_agents_per_formation": N}))


def test_abi_version_matches_header(flib):
    """fenv_abi_version() == the header's FENV_ABI_VERSION (a host program checks this at start)."""
    import re
    src = open(flib.HEADER).read()
    want = int(re.search(r"#define FENV_ABI_VERSION (\d+)", src).group(1))
    assert flib.lib().fenv_abi_version() == want >= 2
    assert flib.lib().ppo_workspace_bytes() >= 16


def test_host_free_rejects_foreign_pointers(flib):
    """fenv_host_free(NULL) is a no-op; a pointer fenv_host_alloc did not hand out (or already
    took back) is rejected with FENV_EINVAL before anything is read from it (no device needed)."""
    import ctypes
    L = flib.lib()
    assert L.fenv_host_free(0, None) == 0
    buf = ctypes.create_string_buffer(1024)
    assert L.fenv_host_free(0, ctypes.cast(ctypes.byref(buf, 512), ctypes.c_void_p)) != 0
    assert b"fenv_host_alloc" in L.fenv_last_error()
    h, d = ctypes.c_void_p(), ctypes.c_void_p()
    assert L.fenv_host_alloc(0, -1, ctypes.byref(h), ctypes.byref(d)) != 0


def test_destroy_null_and_range_args_fail_cleanly(flib):
    """fenv_destroy(NULL) is a no-op; the range queries reject a NULL handle with an error code
    (no device needed)."""
    L = flib.lib()
    assert L.fenv_destroy(None) == 0
    assert L.fenv_get_state_range(None, 0, 1, None, None, None, None, None, None) != 0
    assert L.fenv_metrics_range(None, 0, 1, None, None, None, None) != 0
    assert b"NULL" in L.fenv_last_error()


def test_destroy_of_unknown_handle_is_refused(flib):
    """fenv_destroy checks the library's set of live handles, so a pointer
    that was never created (or was destroyed already) is refused with FENV_EINVAL before any of
    its memory is read -- here a host buffer full of garbage stands in for a freed handle."""
    import ctypes
    L = flib.lib()
    junk = ctypes.create_string_buffer(b"\xff" * 4096)
    assert L.fenv_destroy(ctypes.cast(junk, ctypes.c_void_p)) == -1
    assert b"not a live handle" in L.fenv_last_error()


def test_device_address_lookup(flib):
    """``_lib.device_address``: an array inside a registered host block maps to the block's
    device address plus its offset; unaligned starts, non-contiguous views and arrays outside
    every block map to None, and so does a block mapped for another device than the one asked
    for (host logic only: the block here is a registry entry, no device)."""
    import numpy as np
    base = np.zeros(256, np.float32)
    p = base.ctypes.data
    flib._blocks[p] = (base.nbytes, 0x7000_0000, 1)
    try:
        assert flib.device_address(base).value == 0x7000_0000
        assert flib.device_address(base, "cuda:1").value == 0x7000_0000
        assert flib.device_address(base, "cuda:0") is None            # mapped for device 1
        assert flib.device_address(base[8:40]).value == 0x7000_0000 + 32
        assert flib.device_address(base[1:9]) is None                 # 4-B aligned start
        assert flib.device_address(base[1:9], align=4).value == 0x7000_0000 + 4
        assert flib.device_address(base.reshape(16, 16)[:, :4]) is None  # not C-contiguous
        assert flib.device_address(base.copy()) is None                # another allocation
        assert flib.device_address([1.0, 2.0]) is None
    finally:
        flib._blocks.pop(p, None)
    assert flib.device_address(base) is None


def test_stream_gate_argument_errors(flib):
    """fenv_stream_gate validates its arguments before any HIP call: a NULL flag or a timeout
    outside (0, 60 s] is FENV_EINVAL (no device needed)."""
    import ctypes
    L = flib.lib()
    flag = ctypes.c_void_p(0x1000)
    assert L.fenv_stream_gate(None, 1, 1000, None, None) == -1
    assert b"fenv_stream_gate" in L.fenv_last_error()
    assert L.fenv_stream_gate(flag, 1, 0, None, None) == -1
    assert L.fenv_stream_gate(flag, 1, 60_000_001, None, None) == -1
