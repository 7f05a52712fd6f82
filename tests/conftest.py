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


class Tuning:
    """pb_tune_set from tests: the launchers' kernel-selection / launch-shape parameters, named as
    the library names them ("mg_engine_min_plane") or in the env-style spelling the tests used
    before the table existed ("PB_MG_ENGINE_MIN_PLANE")."""

    def __init__(self, pb):
        self.pb = pb

    @staticmethod
    def name(n):
        return n[3:].lower() if n.startswith("PB_") else n

    def set(self, name, value):
        self.pb.tune_set(self.name(name), int(value))

    setenv = set


@pytest.fixture
def tune():
    import poissbox_amd as pb
    pb.tune_reset()
    yield Tuning(pb)
    pb.tune_reset()
