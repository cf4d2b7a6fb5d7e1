import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "joint-multimodal-transformer-6th-abaw_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


@pytest.fixture(scope="session")
def golden():
    path = os.path.join(REPO, "tests", "golden", "golden.npz")
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}
