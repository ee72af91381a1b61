"""Import helper: the package directory is ``marl-distributedformation_amd/`` (a hyphenated name
Python cannot ``import`` directly); this registers it as ``marl_distributedformation_amd``."""
from __future__ import annotations

import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "marl-distributedformation_amd")
NAME = "marl_distributedformation_amd"


def load():
    mod = sys.modules.get(NAME)
    if mod is not None:
        return mod
    spec = importlib.util.spec_from_file_location(
        NAME, os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[NAME] = mod
    spec.loader.exec_module(mod)
    return mod
