import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running (stress / multi-process)")


def _ensure_built():
    """Build the in-tree native core once per session (seconds; skipped when up to date)."""
    sys.path.insert(0, str(ROOT / "native"))
    import build  # native/build.py

    build.build_core()
    build.build_topo_cli()


_ensure_built()


@pytest.fixture
def fake_store():
    from nanogpu.k8s.fake_apiserver import FakeKubeStore

    return FakeKubeStore()


@pytest.fixture
def tmp_shm(tmp_path):
    """A ledger path in /dev/shm that is removed afterwards."""
    p = Path("/dev/shm") / f"nanogpu-test-{os.getpid()}-{tmp_path.name}"
    yield str(p)
    try:
        p.unlink()
    except FileNotFoundError:
        pass


@pytest.fixture
def cpu_exclusive():
    """Multi-process bench jobs (several ranks, each with busy front-door threads, plus the API
    server and the stand-ins) measure timing-sensitive things; under `pytest -n` they take turns
    (an exclusive lock across the xdist workers) instead of starving each other."""
    import fcntl

    with open("/tmp/nanogpu-tests-cpu-exclusive.lock", "w") as f:
        fcntl.flock(f, fcntl.LOCK_EX)
        try:
            yield
        finally:
            fcntl.flock(f, fcntl.LOCK_UN)
