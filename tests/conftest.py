import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libhbgpu.so on the device)")
    config.addinivalue_line("markers", "slow: larger CPU-side checks")


@pytest.fixture(scope="session")
def ctx():
    from hydrabadger_amd import _lib
    c = _lib.default_context()
    yield c
