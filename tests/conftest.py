import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through the C ABI)")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build the oracle (and, if hipcc is present, the HIP library) once."""
    import __graft_entry__ as g

    g.build()
    yield
