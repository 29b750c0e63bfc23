"""pytest config: registers the `gpu` marker and puts the repo root and the package dir on sys.path.

`-m "not gpu"` runs everywhere (oracle vs golden fixtures, host logic, C-ABI load/export checks,
gloo world_size-2 tests); `-m gpu` runs the HIP parity tests on an MI355X.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "residual-td3-robot-navigation_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP kernels run)")


def golden(name):
    import numpy as np
    return np.load(os.path.join(GOLDEN, name))


@pytest.fixture(scope="session")
def orc():
    from oracle import oracle
    oracle.build()
    return oracle


@pytest.fixture(autouse=True)
def _seeded_torch():
    """Every test draws its unseeded torch inputs from the same stream: reproducible runs."""
    import torch
    torch.manual_seed(0)
    yield
