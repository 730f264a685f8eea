import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run on the GPU box with -m gpu)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session", autouse=True)
def _build_native():
    """Build the in-tree native core once per session (cheap when up to date)."""
    from aiforearth_api_platform_amd import _build

    _build.build_core()
    yield


@pytest.fixture(params=["native", "python"])
def backend(request):
    return request.param


@pytest.fixture
def fresh_config(monkeypatch):
    from aiforearth_api_platform_amd import config as cfgmod

    cfg = cfgmod.Config.load(env={})
    cfgmod.set_config(cfg)
    yield cfg
    cfgmod.set_config(None)
