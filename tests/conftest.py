import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run on the GPU box)")
    config.addinivalue_line("markers", "slow: longer CPU test")


def scene_path(name):
    for ext in (".cgltrace", ".cgltrace.gz"):
        p = os.path.join(GOLDEN, "scenes", name + ext)
        if os.path.exists(p):
            return p
    raise FileNotFoundError(name)


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import py_oracle
    py_oracle.build()
    return py_oracle
