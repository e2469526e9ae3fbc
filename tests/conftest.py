import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT / "packet-process-engine_amd", ROOT / "oracle"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

GOLDEN = ROOT / "tests" / "golden"
NOW = 1_700_000_000


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through the C ABI)")


@pytest.fixture(scope="session")
def golden():
    return dict(np.load(GOLDEN / "golden_v1.npz"))


@pytest.fixture(scope="session")
def ref_hash():
    return dict(np.load(GOLDEN / "ref_tluhash_v1.npz"))
