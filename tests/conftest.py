import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU available")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session", autouse=True)
def _native_build():
    """Incremental in-tree build of the native extensions (no-op when fresh).
    On a GPU box the extensions built here travel with the tree (build/ does
    not): use them as they are instead of rebuilding inside the test run."""
    import glob

    import torch

    from tensorflow_distributed_on_gke_amd import _build

    built = len(glob.glob(os.path.join(ROOT, "tensorflow_distributed_on_gke_amd", "_*.so"))) >= 2
    if not (torch.cuda.is_available() and built):
        _build.build()
    yield
