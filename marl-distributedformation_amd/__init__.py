"""MI355X-native batched formation-control env + policy rollout (drop-in for the reference's
FormationEnv hot path).

Import this package as ``marl_distributedformation_amd`` through :func:`pkgload.load` at the
repo root (the directory name carries a hyphen).
"""
from .config import load_config, Config  # noqa: F401

__all__ = ["FormationEnv", "load_config", "Config", "lib"]


def __getattr__(name):
    # lazy: importing the package must not require a GPU or a built library
    if name == "FormationEnv":
        from .vectorized_env import FormationEnv
        return FormationEnv
    if name == "lib":
        from . import _lib
        return _lib.lib()
    raise AttributeError(name)
