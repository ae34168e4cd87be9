import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs an MI355X (runs the HIP engine)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def built_lib():
    from mpcc_manipulator_amd import _build
    return _build.build()


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import pyoracle
    pyoracle.build()
    return pyoracle
