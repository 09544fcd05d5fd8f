import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gnot-replication_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built libgnot_hip.so")


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if gpu_available():
        return
    skip = pytest.mark.skip(reason="no ROCm GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def mid_case():
    """configs[2] / configs[3] widths (d=256, 8 heads, 8 experts, 4-layer MLPs, one 805-point input
    function), L = 1 block, one 70,000-point mesh, with its float64 (and float32) CPU-oracle output and
    gradients: shared by the headline-size tests (test_gpu_headline.py) and the point-sharded test at
    these widths (test_gpu_shard.py), so the ~2 minutes of oracle work run once per session."""
    from test_gpu_configs import CFG_3D
    from test_gpu_parity import _random_case
    return _random_case(31, dict(CFG_3D, n_attn_layers=1), [70000], [[805]])
