import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libpoissbox_gpu.so)")


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    return np.load(os.path.join(REPO, "tests", "golden", "ref_fixtures.npz"))


@pytest.fixture(scope="session")
def ctx():
    import poissbox_amd as pb
    c = pb.Context(0)
    yield c
    c.destroy()
