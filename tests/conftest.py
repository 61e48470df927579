import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); runs the HIP kernels")
    config.addinivalue_line("markers", "slow: multi-second CPU test")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


def rel_close(got, ref, tol=1e-4):
    """The parity bar for fp32 scores: |got - ref| <= tol * max(1, |ref|), elementwise."""
    import numpy as np
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    err = np.abs(got - ref) / np.maximum(1.0, np.abs(ref))
    return float(err.max()) if err.size else 0.0
