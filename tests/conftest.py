import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); parity tests through the C ABI")
    config.addinivalue_line("markers", "slow: long-running")


def pytest_collection_modifyitems(config, items):
    gpu_ok = None
    for item in items:
        if "gpu" in item.keywords:
            if gpu_ok is None:
                import torch

                gpu_ok = torch.cuda.is_available()
            if not gpu_ok:
                item.add_marker(pytest.mark.skip(reason="no HIP device"))
