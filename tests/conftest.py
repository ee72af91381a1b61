import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and libfenv.so")


@pytest.fixture(scope="session")
def pkg():
    import pkgload
    return pkgload.load()


@pytest.fixture(scope="session")
def venv(pkg):
    from importlib import import_module
    return import_module(pkg.__name__ + ".vectorized_env")


@pytest.fixture(scope="session")
def flib(pkg):
    from importlib import import_module
    return import_module(pkg.__name__ + "._lib")
