import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle_py

    oracle_py.load()
    return oracle_py


@pytest.fixture(scope="session")
def gpu_aligner_factory():
    from crispresso_amd.aligner import GpuAligner
    from crispresso_amd.needle_options import NeedleOptions

    made = []

    def make(options=None):
        a = GpuAligner(0, options or NeedleOptions())
        made.append(a)
        return a

    yield make
    for a in made:
        a.close()
