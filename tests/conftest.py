import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

REFERENCE_DIR = "/root/reference/ProteinBERT"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def reference_modules():
    """The reference model file imports with torch alone."""
    if not os.path.exists(os.path.join(REFERENCE_DIR, "modules.py")):
        pytest.skip("reference not mounted")
    sys.path.insert(0, REFERENCE_DIR)
    try:
        import modules  # type: ignore
    finally:
        sys.path.remove(REFERENCE_DIR)
    return modules
