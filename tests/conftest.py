"""pytest configuration: the `gpu` marker and shared paths.

`-m "not gpu"` (CPU container): oracle vs golden fixtures, host logic (pattern / planner),
C-ABI library load + symbol exports, gloo world_size-2 routing tests.
`-m gpu` (MI355X box): parity of the HIP path against the oracle, through the C ABI.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) — run on the GPU box")


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")
