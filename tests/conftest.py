import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle():
    from oracle.bind import Oracle, build
    build(ref=False)
    return Oracle()


@pytest.fixture(scope="session")
def golden_ops():
    import numpy as np
    return dict(np.load(os.path.join(ROOT, "tests", "golden", "ops_ref.npz")))


@pytest.fixture(scope="session")
def golden_models():
    import numpy as np
    return dict(np.load(os.path.join(ROOT, "tests", "golden", "model_ref.npz")))
