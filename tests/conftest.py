import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line(
        "markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def hip_lib():
    """The product library, loaded for the GPU tests.  Fails loudly when the
    HIP extension is missing (no CPU fallback exists)."""
    import quadiron_amd
    lib = quadiron_amd.lib()
    if lib.qi_gpu_device_count() < 1:
        pytest.fail("no HIP device visible to the product library")
    return lib
