"""Native core under ASan+UBSan and TSan (host code only; no GPU sanitizers on this pool).

native/tests/stress_main.cpp churns a /dev/shm ledger from several threads and a forked
second process while the native HTTP front door answers filter/priorities, then checks
that every device is whole again (SURVEY §4 lesson 5); then drives the native API server
with native bind writers, concurrent patches and a watch stream (no lost update, every event
delivered); then watch-gap deletions against concurrent relist reconciliation; then responses
posted from another thread while the front-door workers park and wake (the mailbox path)."""
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "native"))


@pytest.mark.parametrize("kind,threads,iters", [("plain", 4, 3000), ("asan", 4, 1500), ("tsan", 3, 800)])
def test_native_stress(kind, threads, iters, cpu_exclusive):
    import build

    exe = build.build_stress(kind)
    r = subprocess.run([str(exe), str(threads), str(iters)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "stress ok" in r.stdout and "relist ok" in r.stdout and "handoff ok" in r.stdout
    assert "mailbox ok" in r.stdout and "inline ok" in r.stdout and "frontdoor ok" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "WARNING: ThreadSanitizer" not in r.stderr
