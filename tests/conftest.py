import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    if os.environ.get("HGX_LIB_VARIANT"):   # the suite tests the product library, never an A/B variant
        raise pytest.UsageError("HGX_LIB_VARIANT is set: unset it to run the tests on hypergraphdb_amd/libhgx.so")
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine through the C ABI)")
    config.addinivalue_line("markers", "slow: long CPU-side check")


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle_ctypes
    return oracle_ctypes.lib()
