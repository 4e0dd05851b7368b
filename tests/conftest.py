import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "dfu-multimodal_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


@pytest.fixture(autouse=True)
def _library_default_precision():
    """Every test starts and ends in the library's default forward precision (a test that
    changes it with set_precision cannot leak its mode into the next one)."""
    fn = sys.modules.get("dfu_hip.functional")
    if fn is not None:
        fn.set_precision(fn.DEFAULT_PRECISION)
    yield
    fn = sys.modules.get("dfu_hip.functional")
    if fn is not None:
        fn.set_precision(fn.DEFAULT_PRECISION)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)
