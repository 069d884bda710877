import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

import __graft_entry__ as entry  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libvpx_hip.so on cuda:0)")
    config.addinivalue_line("markers", "slow: full-size (BASELINE.json) configuration")


@pytest.fixture(scope="session")
def pkg():
    return entry.load_package()


@pytest.fixture(scope="session")
def orc():
    return entry.load_oracle()


@pytest.fixture(scope="session")
def abi(pkg):
    return pkg.abi
