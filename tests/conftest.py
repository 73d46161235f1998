import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, TESTS):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs librt_hip.so kernels)")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build librt_hip.so and the oracle if they are missing (hipcc cross-compiles without a GPU)."""
    import __graft_entry__

    lib = os.path.join(ROOT, "cudaraytracer_amd", "librt_hip.so")
    orc = os.path.join(ROOT, "oracle", "build", "liboracle.so")
    if not (os.path.exists(lib) and os.path.exists(orc)):
        __graft_entry__.build()
