import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running test")
    config.addinivalue_line("markers", "no_stream_audit: builds a stream hazard on purpose (skips DLGM_STREAM_AUDIT)")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


def pytest_sessionfinish(session, exitstatus):
    """Leave no /dev/shm checkpoint snapshot tier behind (tests that fail before discarding it)."""
    import glob

    if os.environ.get("PYTEST_XDIST_WORKER"):
        return
    for p in glob.glob("/dev/shm/dlgm-ckpt-*"):
        try:
            os.unlink(p)
        except OSError:
            pass


@pytest.fixture(autouse=True)
def _stream_audit(request):
    """DLGM_STREAM_AUDIT=1: every GPU test runs under the stream-ordering audit (utils/stream_audit.py) and fails
    if any op it issued is not ordered after a conflicting access on another HIP stream, or reuses a freed block
    another stream may still be using. Tests that build such hazards on purpose carry ``no_stream_audit``."""
    from distributed_llm_training_gpu_manager_amd.utils import stream_audit as sa

    if "gpu" not in request.keywords or "no_stream_audit" in request.keywords or \
            not (sa.enabled() or sa.poison_enabled()):
        yield
        return
    import contextlib
    with contextlib.ExitStack() as st:
        if sa.poison_enabled():  # DLGM_POISON_ALLOC=1: uninitialised float allocations read as NaN
            st.enter_context(sa.poison_allocations())
        audit = st.enter_context(sa.stream_audit(stack=True)) if sa.enabled() else None
        yield
    if audit is not None and audit.hazards:
        pytest.fail(audit.report(), pytrace=False)
