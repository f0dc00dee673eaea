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
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu")
    # rank processes decide their hardware-queue count from this before HIP starts (tests/mp_util.py)
    import mp_util

    mp_util.export_device_count()


@pytest.fixture(scope="session")
def built():
    """Build (incrementally) the product library and the oracle once per session."""
    from mscclpp_amd import _build

    _build.build_oracle()
    _build.build_library()
    _build.build_audit()
    _build.build_tests()
    _build.build_diag()
    return True
