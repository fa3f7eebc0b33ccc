"""pytest configuration: `-m gpu` selects tests that need an MI355X; the rest
run on a CPU-only host (multi-process paths use the gloo backend)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X)")
    config.addinivalue_line("markers", "slow: longer-running test")


@pytest.fixture(scope="session", autouse=True)
def _native_built():
    """Build the in-tree extension + CLIs once per session (incremental)."""
    from dpsvm_amd import build

    build.build(clis=True, verbose=False)
    yield


@pytest.fixture(scope="session")
def C():
    from dpsvm_amd._native import load

    return load()


@pytest.fixture(scope="session")
def bin_dir():
    return os.path.join(ROOT, "bin")


def run(cmd, **kw):
    kw.setdefault("capture_output", True)
    kw.setdefault("text", True)
    kw.setdefault("timeout", 600)
    return subprocess.run(cmd, **kw)
