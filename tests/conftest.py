import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")
    config.addinivalue_line("markers", "slow: long-running (large problem sizes)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O

    O.lib()
    return O


@pytest.fixture(scope="session")
def queue():
    import conjugategradient_amd as cga

    n = cga.device_count()
    assert n >= 1, "gpu tests need a HIP device: libcgx sees none"
    q = cga.Queue(0)
    yield q
    q.close()
