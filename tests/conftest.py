import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def main_model():
    from ur3e_amd.model.compiler import load_json, to_ctypes
    md = load_json(os.path.join(REPO, "ur3e_amd", "assets", "main.model.json"))
    return md, to_ctypes(md)


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    return dict(np.load(os.path.join(REPO, "tests", "golden", "reference_golden.npz")))
