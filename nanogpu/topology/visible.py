"""How many GPUs a process started now would see, without initialising HIP.

bench.py's launcher asks this before it starts one rank per GPU: nothing in the launching
process may touch the GPU (a process that has initialised HIP must not be replaced, and its
children would inherit nothing useful). The count comes from the KFD sysfs topology the
native reader walks (`_native.discover_topology(root, use_amdsmi=False)`: one entry per
device HIP enumerates, so a CPX-partitioned MI355X counts 8), narrowed by the runtime's
visibility variables the way ROCm applies them: `ROCR_VISIBLE_DEVICES` selects among the
agents first, then `HIP_VISIBLE_DEVICES` (or its alias `CUDA_VISIBLE_DEVICES`) indexes
into what is left, then `GPU_DEVICE_ORDINAL`.
"""
from __future__ import annotations

import json
import os
from typing import Mapping

VISIBILITY_VARS = ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "GPU_DEVICE_ORDINAL")


def sysfs_gpu_count(sysfs_root: str = "") -> int:
    """Devices the KFD topology under `sysfs_root` ("" = the live /sys) lists; 0 if none or
    if the native reader is missing."""
    try:
        from nanogpu.native import core

        host = json.loads(core().discover_topology(sysfs_root, False))
    except Exception:
        return 0
    return len(host.get("gpus", []))


def _narrow(n: int, spec: str | None) -> int:
    """Devices left of `n` after one visibility list. An index past the end, or any entry
    after it, hides the rest (the runtime stops at the first invalid ordinal); a UUID
    (`GPU-...`) counts as one device. Set but empty reads as unset: HIP's runtime flag
    defaults to "" meaning every device (this build container exports HIP_VISIBLE_DEVICES=)."""
    if spec is None or not spec.strip():
        return n
    spec = spec.strip()
    seen: set[str] = set()
    for tok in (t.strip() for t in spec.split(",")):
        if not tok:
            break
        if tok.lstrip("-").isdigit():
            i = int(tok)
            if i < 0 or i >= n:
                break
        if tok in seen:
            break
        seen.add(tok)
    return min(n, len(seen))


def visible_gpu_count(sysfs_root: str = "", env: Mapping[str, str] | None = None) -> int:
    env = os.environ if env is None else env
    n = sysfs_gpu_count(sysfs_root)
    rocr = env.get("ROCR_VISIBLE_DEVICES")
    hip = env.get("HIP_VISIBLE_DEVICES", env.get("CUDA_VISIBLE_DEVICES"))
    for spec in (rocr, hip, env.get("GPU_DEVICE_ORDINAL")):
        n = _narrow(n, spec)
    return n
