import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "query-engine_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libqeh.so on cuda:0)")


@pytest.fixture(scope="session")
def ctx():
    import qe_hip
    c = qe_hip.Context(0)
    yield c
    c.close()
