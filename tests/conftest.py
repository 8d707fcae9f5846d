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


@pytest.fixture(params=["sweep", "bands"])
def mb_path(request, monkeypatch):
    """The two multi-band implementations (mcs_capi.cpp prepare_sweep): the band pass + blend
    kernels (the default) and the fused sweep kernel (mcs_sweep.hip, opt-in MCS_MB_SWEEP=1; plans
    it does not take keep the band pass).  Read when a plan prepares its tables."""
    monkeypatch.setenv("MCS_MB_SWEEP", "1" if request.param == "sweep" else "0")
    return request.param


def check_mb_path(stats, path, sweep_expected=True):
    """The plan took the multi-band path the test asked for."""
    if path == "bands":
        assert stats["mb_sweep_strips"] == 0, stats
    elif sweep_expected:
        assert stats["mb_sweep_strips"] > 0 and stats["mb_bands"] == 0, stats
