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
    config.addinivalue_line("markers", "record_path: bitwise comparisons between runs or paths: the backward "
                                       "takes the deterministic record path (bwd_atomic=0) whatever the default")


@pytest.fixture(autouse=True)
def _record_path(request):
    """Tests marked record_path compare backward results bit for bit between runs or code paths; the atomic
    backward (the "bwd_atomic" option) adds in the hardware's order, so they pin the deterministic record
    path (render_bwd records + gauss_reduce) for their duration."""
    if request.node.get_closest_marker("record_path") is None:
        yield
        return
    from gaussian_splatting_amd import _lib

    with _lib.options(bwd_atomic=0):
        yield


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
