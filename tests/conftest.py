import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X) and libpa_hip.so")


@pytest.fixture(scope="session")
def pamd():
    import pamd as m
    return m


@pytest.fixture(scope="session")
def O():
    import pa_oracle
    return pa_oracle
