"""Shared pytest configuration.

Markers: ``gpu`` tests need an MI355X (run on the GPU box with ``-m gpu``);
everything else runs on the CPU-only container.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an AMD Instinct MI355X (gfx950)")
    config.addinivalue_line("markers", "slow: long-running (large arrays)")


# The full-size parity tests of BASELINE's configurations against the
# reference's hashes run first, so that a GPU run cut short (pytest -x, a
# time limit) has still pinned every BASELINE config before the fuzz loops.
_FIRST = ("test_golden_baseline_configs", "test_golden_1024_full_array", "test_golden_1024_slab")


def pytest_collection_modifyitems(session, config, items):
    def rank(item):
        name = item.originalname or item.name
        return _FIRST.index(name) if name in _FIRST else len(_FIRST)
    items.sort(key=rank)  # stable: everything else keeps its order


@pytest.fixture(scope="session")
def restatement():
    import oracle
    if oracle.restatement is None:
        oracle.build(with_reference=False)
        oracle.reload()
    return oracle.restatement


@pytest.fixture(scope="session")
def reference():
    """The reference's own CPU zfp 0.5.0 (oracle/_ref), or skip if it was never built."""
    import oracle
    if oracle.reference is None:
        pytest.skip("oracle/_ref/libzfp_ref.so not built (needs /root/reference)")
    return oracle.reference


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but no GPU is visible")
    return torch.device("cuda:0")
