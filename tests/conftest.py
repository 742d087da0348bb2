import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C-ABI)")


@pytest.fixture(scope="session")
def kat():
    with np.load(os.path.join(GOLDEN, "kat.npz")) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def traj():
    with np.load(os.path.join(GOLDEN, "traj.npz")) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def oracle_c():
    from oracle import oracle_c as oc
    oc.lib()
    return oc
