import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run via gpurun)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session", autouse=True)
def library_is_heads():
    """Every test that touches libccrec_hip.so runs on a binary compiled from THIS tree's
    csrc/ + include/ (cc_build_id() == buildid.tree_build_id()); a stale library fails the run."""
    from cubecobrarecommender_amd import _lib
    if os.path.exists(_lib.LIB_PATH):
        _lib.check_build_id()


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")
