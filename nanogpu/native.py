"""Loader for the in-tree native extensions.

`_native` (C++ core) is mandatory: the scheduler has no pure-Python allocation path, so a
missing build fails loudly instead of silently falling back. `_probe` (HIP, gfx950) is
needed only by the node agent's calibration and GPU tests; `probe(required=True)` raises
on a GPU host where it is missing.
"""
from __future__ import annotations

import importlib
import os
from types import ModuleType

_BUILD_HINT = "build it in-tree with `python native/build.py` (or __graft_entry__.build())"


def core() -> ModuleType:
    try:
        return importlib.import_module("nanogpu._native")
    except ImportError as e:  # pragma: no cover - exercised only on broken installs
        if os.environ.get("NANOGPU_AUTOBUILD", "1") == "1":
            from pathlib import Path
            import subprocess
            import sys

            root = Path(__file__).resolve().parent.parent
            subprocess.run([sys.executable, str(root / "native" / "build.py"), "--no-hip"], check=True)
            return importlib.import_module("nanogpu._native")
        raise ImportError(f"nanogpu._native is not built; {_BUILD_HINT}") from e


def _hip_runtime_first() -> None:
    """PyTorch-ROCm bundles its own libamdhip64.so.7 with the same SONAME as /opt/rocm's.
    Whichever loads first serves the whole process, and torch's CUDA/HIP API fails on a
    foreign runtime. So torch (when installed) is imported before the probe, and the
    probe's kernels run on torch's runtime (verified on MI355X: tests/test_gpu.py)."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def probe(required: bool = False, build: bool = False) -> ModuleType | None:
    _hip_runtime_first()
    try:
        return importlib.import_module("nanogpu._probe")
    except ImportError as e:
        if build and os.environ.get("NANOGPU_AUTOBUILD", "1") == "1":
            from pathlib import Path
            import subprocess
            import sys

            root = Path(__file__).resolve().parent.parent
            r = subprocess.run([sys.executable, str(root / "native" / "build.py")], capture_output=True, text=True)
            if r.returncode == 0:
                return importlib.import_module("nanogpu._probe")
        if required:
            raise ImportError(f"nanogpu._probe (HIP gfx950 kernels) is not built; {_BUILD_HINT}") from e
        return None
