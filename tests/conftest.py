import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# Scratch buffers 0xff-filled, outputs NaN-filled before every native call (_C.py): reads of
# memory no kernel wrote show up as failures rather than depending on the allocator.
os.environ.setdefault("GSR_POISON", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built libgsr.so")
    config.addinivalue_line("markers", "slow: long-running (full-size configs)")


def pytest_collection_modifyitems(config, items):
    # GPU tests need a visible HIP device; on a CPU-only host they are reported as skipped
    # unless explicitly selected with -m gpu (then they fail loudly instead).
    import torch

    selected = config.getoption("-m") or ""
    if torch.cuda.is_available() or "gpu" in selected.replace("not gpu", ""):
        return
    skip = pytest.mark.skip(reason="no HIP device on this host")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)
