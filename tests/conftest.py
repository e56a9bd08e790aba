import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "svt-av1_pro-anchor-v2.1.0-_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")
    config.addinivalue_line("markers", "slow: longer CPU test")
    # torch bundles its own HIP runtime and must initialize the device before libsvtgpu's runtime does (the order
    # bench.py uses), or torch reports no GPU: do it before collection, where a test module could touch the device
    if os.path.exists("/dev/kfd"):
        try:
            import torch
            if torch.cuda.is_available():
                torch.cuda.init()
        except ImportError:
            pass


@pytest.fixture(scope="session", autouse=True)
def _torch_hip_first(request):
    """torch bundles its own HIP runtime; it must initialize the device before libsvtgpu's runtime does (the
    order bench.py uses), or torch reports no GPU.  Only when GPU tests are selected."""
    if any(item.get_closest_marker("gpu") for item in request.session.items):
        try:
            import torch
            if torch.cuda.is_available():
                torch.cuda.init()
        except ImportError:
            pass
    yield
