import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import oracle

    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def gpu():
    """The native library on a visible HIP device (GPU tests only)."""
    from gfa2network_amd import _native

    _native.load()
    if _native.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests need the MI355X")
    return _native
