import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP kernels); run with -m gpu")
    config.addinivalue_line("markers", "slow: longer CPU test")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(autouse=True)
def _bounds_check(request):
    """P2P_BOUNDS_CHECK=1 (with P2P_LIB = the P2P_BOUNDS_ASSERT build, csrc/bounds.h): after
    every GPU test, no kernel may have taken an out-of-range store / load index."""
    yield
    if os.environ.get("P2P_BOUNDS_CHECK") != "1" or "gpu" not in request.node.keywords:
        return
    import torch
    from p2p_pytorch_amd import _native
    if not _native.load():
        return
    on, count, site, idx, limit = torch.ops.p2p.oob_counts(True)
    assert on == 1, "P2P_BOUNDS_CHECK=1 needs the P2P_BOUNDS_ASSERT build (P2P_LIB)"
    assert count == 0, f"{count} out-of-range indices (largest site id {site}, last index {idx}, limit {limit})"
