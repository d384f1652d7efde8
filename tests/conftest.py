import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built libnlot.so")
    config.addinivalue_line("markers", "slow: long CPU-oracle runs")


@pytest.fixture(scope="session")
def artefact():
    from nlotrajectories_amd.nn import MlpWeights

    return MlpWeights.artefact()


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    return dict(np.load(os.path.join(ROOT, "tests", "golden", "mlp_artefact_golden.npz")))
