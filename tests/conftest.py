import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")
    config.addinivalue_line("markers", "slow: long-running test")


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no GPU available")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


_GPU_FAULT_SIGNS = ("illegal memory access", "Memory access fault", "hipErrorIllegalAddress", "HSA_STATUS_ERROR")


@pytest.hookimpl(hookwrapper=True)
def pytest_runtest_makereport(item, call):
    """A GPU fault poisons the HIP context for every later test: end the session at the first one (even
    without -x), so nothing else runs on a faulted device."""
    outcome = yield
    rep = outcome.get_result()
    if rep.failed and call.excinfo is not None and any(s in str(call.excinfo.value) for s in _GPU_FAULT_SIGNS):
        pytest.exit(f"GPU fault in {item.nodeid}: stopping the session", returncode=98)
