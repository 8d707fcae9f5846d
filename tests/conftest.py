import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


@pytest.fixture(scope="session", autouse=True)
def _built_libraries():
    """Build the oracle (test infrastructure) and libmcs once per session if stale."""
    from oracle import oracle
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        oracle.build()
    from multicamera_stitching_amd import build
    build.build()
    yield
