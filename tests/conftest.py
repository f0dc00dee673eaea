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
    config.addinivalue_line("markers", "reference_kernel: runs the reference's own multi-rank kernel (no spin bound)")
    # rank processes decide their hardware-queue count from this before HIP starts (tests/mp_util.py)
    import mp_util

    mp_util.export_device_count()


def pytest_collection_modifyitems(config, items):
    """The reference's own multi-rank kernels spin without a bound (their device asserts compile out in
    release builds), so a wedged rank there can only end its worker process: run them after
    everything else, so such a failure cannot keep the rest of the suite from running under -x."""
    items.sort(key=lambda it: it.get_closest_marker("reference_kernel") is not None)


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
