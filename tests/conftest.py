import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "thyroid-nodule-image-segmentation-unet-ddti_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run on the GPU box)")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(autouse=True)
def _reset_schedule_options():
    """Runtimes are cached per device and network configuration (unet_hip.runtime), so a
    schedule option a test sets would otherwise leak into every later test of that
    configuration: restore every cached runtime's options after each test."""
    yield
    rtmod = sys.modules.get("unet_hip.runtime")
    if rtmod is not None:
        for rt in list(rtmod._RUNTIMES.values()):
            rt.reset_options()
