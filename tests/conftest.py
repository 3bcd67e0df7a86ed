import importlib.util
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def load_golden(name):
    path = os.path.join(GOLDEN, name + ".npz")
    if not os.path.exists(path):
        pytest.skip(f"golden fixture {name} not generated")
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def pkg():
    """The product package (directory rag-cobweb_amd/, imported as rag_cobweb_amd)."""
    import cobweb_pkg
    return cobweb_pkg.load()


@pytest.fixture(autouse=True)
def _categorize_list_paths(monkeypatch):
    """Basic's path choice (cwq_api.hip categorize_impl) is measured at run time: a call may go
    straight to the exact lazy replay instead of the list paths.  The tests that check a
    particular resolution path (counting, replay, two-level, DENSE) pin the list paths; the
    tests of the automatic choice (tests/test_gpu_cut.py) clear this themselves."""
    monkeypatch.setenv("CWQ_CAT_DIRECT", "0")
