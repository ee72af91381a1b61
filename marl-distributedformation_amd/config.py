"""Config keys of the reference (cfg/config.yaml:2-7) with hydra-style ``key=value`` overrides.

The reference reads its config through ``@hydra.main(config_path="cfg", config_name="config")``
(vectorized_env.py:112).  hydra/omegaconf are not part of this build; this module loads the same
YAML (PyYAML, SafeLoader) and applies the same CLI override syntax (README.md:18,21), returning
an attribute-access object with the same key names.
"""
from __future__ import annotations

import os
from types import SimpleNamespace
from typing import Iterable

import yaml

DEFAULT_CFG = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cfg", "config.yaml")

# cfg/config.yaml:2-7 (the reference's keys and defaults)
DEFAULTS = {
    "name": "default",
    "num_formation": 1000,
    "num_agents_per_formation": 5,
    "share_reward_ratio": 0.25,
    "goal_in_obs": True,
}


class Config(SimpleNamespace):
    def to_dict(self) -> dict:
        return dict(vars(self))

    def get(self, key, default=None):
        return getattr(self, key, default)


def _coerce(text: str):
    v = yaml.safe_load(text)
    return v


def load_config(path: str | None = None, overrides: Iterable[str] = ()) -> Config:
    """Load ``path`` (default: the packaged cfg/config.yaml) and apply ``key=value`` overrides.

    Unknown keys are accepted with ``+key=value`` (hydra's append syntax) or plain ``key=value``.
    """
    data = dict(DEFAULTS)
    p = path or DEFAULT_CFG
    if os.path.exists(p):
        with open(p) as fh:
            loaded = yaml.safe_load(fh) or {}
        if not isinstance(loaded, dict):
            raise ValueError(f"{p}: top level must be a mapping")
        data.update(loaded)
    for ov in overrides:
        if "=" not in ov:
            raise ValueError(f"override {ov!r} is not key=value")
        k, v = ov.split("=", 1)
        k = k.lstrip("+").strip()
        if not k:
            raise ValueError(f"override {ov!r} has an empty key")
        data[k] = _coerce(v)
    cfg = Config(**data)
    validate(cfg)
    return cfg


MAX_AGENTS = 1 << 24  # include/fenv.h FENV_MAX_AGENTS


def validate(cfg) -> None:
    F = int(getattr(cfg, "num_formation"))
    N = int(getattr(cfg, "num_agents_per_formation"))
    if F < 1:
        raise ValueError("num_formation must be >= 1")
    if not 1 <= N <= MAX_AGENTS:
        raise ValueError(f"num_agents_per_formation must be in [1, {MAX_AGENTS}]")
    s = float(getattr(cfg, "share_reward_ratio", 0.25))
    if not 0.0 <= s <= 0.5:
        raise ValueError("share_reward_ratio must be in [0, 0.5] (simulate.py:28)")


def as_config(cfg) -> Config:
    """Accept a Config, a dict, an OmegaConf-like or SimpleNamespace object."""
    if isinstance(cfg, Config):
        return cfg
    if isinstance(cfg, dict):
        d = dict(DEFAULTS)
        d.update(cfg)
        return Config(**d)
    d = dict(DEFAULTS)
    for k in list(DEFAULTS) + ["seed", "device", "reset_mode", "max_steps"]:
        if hasattr(cfg, k):
            d[k] = getattr(cfg, k)
    return Config(**d)
