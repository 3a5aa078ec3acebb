import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


def tol_ok(got, ref, rtol=1e-6):
    """North-star parity bar: |got - ref| <= rtol * max(|ref|, 1)."""
    import numpy as np
    got, ref = np.asarray(got, dtype=float), np.asarray(ref, dtype=float)
    return np.abs(got - ref) <= rtol * np.maximum(np.abs(ref), 1.0)
