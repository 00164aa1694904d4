import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device")


@pytest.fixture(scope="session")
def gpu():
    """Fails (never skips) when the HIP path cannot run: a gpu-marked test
    that passes without the device would be a silent fallback."""
    import infinicache_amd as ia
    if not ia.device_ok(0):
        pytest.fail("no usable gfx950 device (rsgpu_device_ok(0) == 0)")
    return 0
