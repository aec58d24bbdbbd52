import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _adipose_pkg  # noqa: E402,F401  (registers `adipose_amd`)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(autouse=True, scope="session")
def _native_option_overrides():
    """ADP_TEST_OPTS="name=value,..." runs the whole session with those native options set (the validation of an
    opt-in kernel form under every test before it becomes a default, e.g. tools/gpu_check.sh)."""
    spec = os.environ.get("ADP_TEST_OPTS", "")
    if spec:
        from adipose_amd import ops
        for kv in spec.split(","):
            if kv:
                ops.set_option(kv.split("=")[0], int(kv.split("=")[1]))
    yield
