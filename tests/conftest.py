import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "6d-pose-estimation_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    d = os.path.join(REPO, "tests", "golden")
    return {
        "pose_loss": np.load(os.path.join(d, "pose_loss.npz")),
        "add_loss": np.load(os.path.join(d, "add_loss.npz")),
    }
