"""SB3-layout checkpoint zips: save, load and the CheckpointCallback schedule.

The reference trains with ``CheckpointCallback(save_freq=10, save_path=f'{this_dir}/logs/{cfg.name}/')``
(vectorized_env.py:124) and plays back the newest ``rl_model_{num_timesteps}_steps.zip``
(visualize_policy.py:29-35) through ``PPO.load``.  stable-baselines3 is not installed here, so
this module writes and reads the SB3 2.x ``save_to_zip_file`` layout itself:

    data                        JSON: the model's hyper-parameters / counters
    policy.pth                  torch.save(policy.state_dict())  (SB3 parameter names)
    policy.optimizer.pth        torch.save(Adam.state_dict()) over the 13 SB3 tensors
    pytorch_variables.pth       torch.save({})
    _stable_baselines3_version  text
    system_info.txt             text

Loading reads ``policy.pth`` with ``torch.load(weights_only=True)`` only (no pickle
execution), so zips written by real SB3 should load here too (unverified: no SB3-written zip
exists here).  Zips written here carry the same entry
names and tensors.  SB3's ``data`` entries for ``policy_class``, ``observation_space`` and
``action_space`` are cloudpickled SB3 / gymnasium objects; round 4 writes them as the pickles
cloudpickle would (``sb3_pickle.py``: the policy class by reference, the reference's two
``Box`` spaces), so the reference's own playback, ``PPO.load(checkpoint_path)`` with no
``custom_objects`` (visualize_policy.py:35), should have what it needs (designed for, not run:
SB3 is absent).  The Adam state's param group
is written with SB3's optimizer settings (non-capturable Adam), so ``set_parameters`` loads it
on any device.  Parity against SB3 itself: unpinned (SB3 and gymnasium absent).
"""
from __future__ import annotations

import io
import json
import os
import platform
import zipfile

import torch

from . import sb3_pickle

SB3_VERSION = "2.3.2"  # the version string written into _stable_baselines3_version

# SB3 ActorCriticPolicy.parameters() order (own Parameter first, then submodules): the index
# order of the optimizer state.  Names as in include/fenv.h / policy.PARAM_SPECS.
SB3_PARAM_ORDER = [
    "log_std",
    "mlp_extractor.policy_net.0.weight", "mlp_extractor.policy_net.0.bias",
    "mlp_extractor.policy_net.2.weight", "mlp_extractor.policy_net.2.bias",
    "mlp_extractor.value_net.0.weight", "mlp_extractor.value_net.0.bias",
    "mlp_extractor.value_net.2.weight", "mlp_extractor.value_net.2.bias",
    "action_net.weight", "action_net.bias",
    "value_net.weight", "value_net.bias",
]

# the param-group settings of the Adam SB3's ActorCriticPolicy builds (torch defaults, eps 1e-5
# set by the policy): a saved group carries them so that SB3 loads it as its own
_SB3_ADAM_GROUP = {"weight_decay": 0, "amsgrad": False, "maximize": False, "foreach": None,
                   "capturable": False, "differentiable": False, "fused": None}


def _tensor_bytes(obj) -> bytes:
    buf = io.BytesIO()
    torch.save(obj, buf)
    return buf.getvalue()


def _state_to_cpu(sd: dict) -> dict:
    return {k: torch.as_tensor(v).detach().to("cpu", torch.float32).clone() for k, v in sd.items()}


def optimizer_state_from_flat(shapes: list[tuple[str, tuple]], opt_state: dict) -> dict:
    """Re-express a torch Adam state over ONE flat parameter (ppo.PPO) as SB3's Adam state over
    the 13 policy tensors (same step count and moments, sliced per tensor)."""
    st = opt_state.get("state", {}).get(0, {})
    groups = opt_state.get("param_groups", [{}])
    offs, o = {}, 0
    for name, shp in shapes:
        n = 1
        for s in shp:
            n *= int(s)
        offs[name] = (o, n, tuple(shp))
        o += n
    state = {}
    for i, name in enumerate(SB3_PARAM_ORDER):
        if not st:
            break
        a, n, shp = offs[name]
        state[i] = {"step": torch.as_tensor(st["step"]).detach().cpu().clone(),
                    "exp_avg": st["exp_avg"][a:a + n].detach().cpu().reshape(shp).clone(),
                    "exp_avg_sq": st["exp_avg_sq"][a:a + n].detach().cpu().reshape(shp).clone()}
    g = {k: v for k, v in groups[0].items() if k != "params"}
    g.update(_SB3_ADAM_GROUP)
    g["params"] = list(range(len(SB3_PARAM_ORDER)))
    return {"state": state, "param_groups": [g]}


def optimizer_state_to_flat(shapes: list[tuple[str, tuple]], opt_state: dict | None,
                            device) -> dict | None:
    """Inverse of :func:`optimizer_state_from_flat`: SB3's Adam state over the 13 policy tensors
    -> {step, exp_avg, exp_avg_sq} over the flat parameter (None if the state is absent,
    empty or does not match the policy's shapes)."""
    if not opt_state or not isinstance(opt_state.get("state"), dict) or not opt_state["state"]:
        return None
    st = opt_state["state"]
    total = 0
    for _, shp in shapes:
        n = 1
        for s in shp:
            n *= int(s)
        total += n
    avg = torch.zeros(total, dtype=torch.float32)
    sq = torch.zeros(total, dtype=torch.float32)
    offs, o = {}, 0
    for name, shp in shapes:
        n = 1
        for s in shp:
            n *= int(s)
        offs[name] = (o, n, tuple(shp))
        o += n
    step = None
    for i, name in enumerate(SB3_PARAM_ORDER):
        e = st.get(i) if i in st else st.get(str(i))
        if not isinstance(e, dict) or "exp_avg" not in e or "exp_avg_sq" not in e:
            return None
        a, n, shp = offs[name]
        ea, es = torch.as_tensor(e["exp_avg"]), torch.as_tensor(e["exp_avg_sq"])
        if tuple(ea.shape) != shp or tuple(es.shape) != shp:
            return None
        avg[a:a + n] = ea.reshape(-1).float()
        sq[a:a + n] = es.reshape(-1).float()
        step = torch.as_tensor(e.get("step", 0)).float().reshape(())
    dev = torch.device(device)
    return {"step": step.to(dev), "exp_avg": avg.to(dev), "exp_avg_sq": sq.to(dev)}


def plain_hyperparameters(data: dict, config_cls) -> dict:
    """The fields of dataclass ``config_cls`` found in an SB3 ``data`` dict, skipping values SB3
    stored as cloudpickled objects (``{":type:": ..., ":serialized:": ...}``, e.g. the
    clip_range / learning_rate schedules) and values whose type does not match the field."""
    out = {}
    for k, f in config_cls.__dataclass_fields__.items():
        if k not in data:
            continue
        v = data[k]
        if isinstance(v, dict):
            continue
        want = type(f.default)
        if want is bool:
            if isinstance(v, bool):
                out[k] = v
        elif want is int:
            if isinstance(v, int) and not isinstance(v, bool):
                out[k] = v
        elif want is float:
            if isinstance(v, (int, float)) and not isinstance(v, bool):
                out[k] = float(v)
    return out


def save_sb3_zip(path: str, state_dict: dict, *, num_timesteps: int, data: dict | None = None,
                 optimizer_state: dict | None = None) -> str:
    """Write an SB3-layout model zip; returns ``path`` (".zip" appended if missing, as SB3)."""
    if not path.endswith(".zip"):
        path += ".zip"
    missing = [k for k in SB3_PARAM_ORDER if k not in state_dict]
    if missing:
        raise KeyError(f"state_dict lacks SB3 parameters {missing}")
    obs_dim = int(state_dict["mlp_extractor.policy_net.0.weight"].shape[1])
    act_dim = int(state_dict["action_net.weight"].shape[0])
    d = sb3_pickle.sb3_opaque_entries(obs_dim, act_dim)
    d.update({"num_timesteps": int(num_timesteps), "_total_timesteps": int(num_timesteps),
              "policy_kwargs": {}})
    d.update(data or {})
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    # the partial file's name must not look like a checkpoint to latest_checkpoint's rule
    tmp = os.path.join(os.path.dirname(os.path.abspath(path)), f".partial-{os.getpid()}.zip")
    with zipfile.ZipFile(tmp, "w") as z:
        z.writestr("data", json.dumps(d, indent=4, sort_keys=False))
        z.writestr("policy.pth", _tensor_bytes(_state_to_cpu(state_dict)))
        if optimizer_state is not None:
            z.writestr("policy.optimizer.pth", _tensor_bytes(optimizer_state))
        z.writestr("pytorch_variables.pth", _tensor_bytes({}))
        z.writestr("_stable_baselines3_version", SB3_VERSION)
        z.writestr("system_info.txt",
                   f"- OS: {platform.platform()}\n- Python: {platform.python_version()}\n"
                   f"- PyTorch: {torch.__version__}\n- Stable-Baselines3: {SB3_VERSION}\n")
    os.replace(tmp, path)
    return path


def load_sb3_zip(path: str, with_optimizer: bool = False):
    """(policy state_dict on CPU, data dict[, optimizer state dict or None]) from an SB3 model
    zip -- ours or SB3's.

    ``policy.pth`` (and ``policy.optimizer.pth`` when asked) are deserialised with
    ``torch.load(weights_only=True)`` only; ``data`` is parsed as JSON and pickled entries are
    left as their JSON stubs.  An optimizer entry the safe loader refuses is reported as None."""
    with zipfile.ZipFile(path) as z:
        names = set(z.namelist())
        if "policy.pth" not in names:
            raise ValueError(f"{path}: no policy.pth (not an SB3 model zip)")
        sd = torch.load(io.BytesIO(z.read("policy.pth")), map_location="cpu", weights_only=True)
        data = json.loads(z.read("data").decode()) if "data" in names else {}
        opt = None
        if with_optimizer and "policy.optimizer.pth" in names:
            try:
                opt = torch.load(io.BytesIO(z.read("policy.optimizer.pth")), map_location="cpu",
                                 weights_only=True)
            except Exception:
                opt = None
    if with_optimizer:
        return dict(sd), data, opt
    return dict(sd), data


def checkpoint_name(num_timesteps: int, prefix: str = "rl_model") -> str:
    """SB3 CheckpointCallback file name: ``{prefix}_{num_timesteps}_steps.zip``."""
    return f"{prefix}_{int(num_timesteps)}_steps.zip"


def latest_checkpoint(directory: str) -> str:
    """The newest checkpoint in ``directory``, chosen as visualize_policy.py:33-34 does: among the
    files whose name contains "rl_model", the one with the largest ``int(name.split("_")[-2])``."""
    files = [f for f in os.listdir(directory) if "rl_model" in f and f.endswith(".zip")]
    if not files:
        raise FileNotFoundError(f"no rl_model_*_steps.zip in {directory}")
    return os.path.join(directory, max(files, key=lambda x: int(x.split("_")[-2].split(".")[0])))


class CheckpointCallback:
    """SB3 ``CheckpointCallback(save_freq, save_path, name_prefix="rl_model")``.

    SB3 calls ``_on_step`` once per vectorised env step inside ``collect_rollouts`` and saves
    whenever ``n_calls % save_freq == 0``, naming the file by the model's ``num_timesteps`` at that
    moment (already counting that step).  :meth:`on_steps` replays that schedule for a rollout of
    ``n`` env steps collected in one launch; the fused collector only exposes the policy at the
    rollout boundary, so every save due inside a rollout is written at its end with that step's
    ``num_timesteps`` (with the reference's save_freq=10 = n_steps the two coincide)."""

    def __init__(self, save_freq: int, save_path: str, name_prefix: str = "rl_model",
                 verbose: int = 0):
        if save_freq < 1:
            raise ValueError("save_freq must be >= 1")
        self.save_freq = int(save_freq)
        self.save_path = save_path
        self.name_prefix = name_prefix
        self.verbose = verbose
        self.n_calls = 0
        self.saved: list[str] = []

    def on_steps(self, model, n: int, num_envs: int) -> list[str]:
        """Advance by a rollout of ``n`` env steps of ``num_envs`` agents that has just been
        collected (``model.num_timesteps`` already counts it); save as SB3 would have."""
        out = []
        t_end = int(model.num_timesteps)
        for s in range(1, int(n) + 1):
            self.n_calls += 1
            if self.n_calls % self.save_freq == 0:
                out.append(self._save(model, t_end - (int(n) - s) * int(num_envs)))
        return out

    def _save(self, model, num_timesteps: int) -> str:
        path = os.path.join(self.save_path, checkpoint_name(num_timesteps, self.name_prefix))
        model.save(path, num_timesteps=num_timesteps)
        self.saved.append(path)
        if self.verbose:
            print(f"Saving model checkpoint to {path}")
        return path

    __call__ = on_steps
