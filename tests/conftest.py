import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")


@pytest.fixture(scope="session")
def hiplib():
    """Build (if stale) and load the in-tree HIP library; no fallback."""
    from xtddft_amd import build, _capi
    build.build()
    return _capi.lib()
