import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); runs the HIP kernels through the C ABI")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.load()
    return O


@pytest.fixture(scope="session")
def gpu():
    """Skip-free GPU guard: -m gpu tests must fail loudly when the HIP path is unavailable."""
    import cuda_iblb_11_amd as P
    n = P.device_count()
    assert n > 0, "no HIP device visible: the -m gpu tests need an MI355X"
    return P
