import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "alphazero-chess_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


# Bind libaz to the /opt/rocm HIP runtime it is built for before anything imports torch
# (torch bundles a libamdhip64.so.7 with the same SONAME).
try:
    import azchess  # noqa: F401,E402
except ImportError:
    pass


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libaz on cuda:0)")


def gpu_available():
    try:
        import azchess._lib as L
        import ctypes
        n = ctypes.c_int(0)
        L.lib.az_device_count(ctypes.byref(n))
        return n.value > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def require_gpu():
    if not gpu_available():
        pytest.fail("GPU test on a machine without a GPU (libaz reports 0 devices)")
    return True
