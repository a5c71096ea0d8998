import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# torch bundles its own libamdhip64.so.7 (same soname as /opt/rocm's): load it
# before libhbgpu.so so the whole test process runs on ONE HIP runtime, as
# bench.py does (torch first).  Loading libhbgpu.so first made torch's CUDA
# unavailable and silently skipped the device-resident (torch) tests.
try:
    import torch  # noqa: F401
except ImportError:  # CPU-only environments without torch still run the oracle tests
    torch = None


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libhbgpu.so on the device)")
    config.addinivalue_line("markers", "slow: larger CPU-side checks")


@pytest.fixture(scope="session")
def ctx():
    from hydrabadger_amd import _lib
    c = _lib.default_context()
    yield c


@pytest.fixture(autouse=True)
def _default_context_left_clean(request):
    """A GPU test must not leave a sticky device error (or a pending HIP
    error) on the shared default context: the next test's synchronising
    call would report it.  Checked after every gpu-marked test that used it."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    from hydrabadger_amd import _lib
    if _lib._default is None:
        return
    rc = _lib.lib().hbg_sync(_lib._default.h)
    assert rc == _lib.HBG_OK, f"{request.node.nodeid} left device error {rc} on the default context"
