"""In-container side of a fractional MI355X grant (import it first, e.g. from sitecustomize).

The device plugin passes the grant through the environment (plugin.py):
  HSA_CU_MASK               spatial share, applied by ROCr itself when queues are created;
  NANO_GPU_MEMORY_FRACTION  HBM budget as a fraction of the device, applied here to the
                            PyTorch caching allocator (cooperative: a process that
                            bypasses the allocator is not capped).
"""
from __future__ import annotations

import os


def grant() -> dict:
    env = os.environ
    return {"devices": env.get("NANO_GPU_DEVICES", ""), "percent": int(env.get("NANO_GPU_PERCENT", "0") or 0),
            "cu_mask": env.get("HSA_CU_MASK", ""), "memory_mib": int(env.get("NANO_GPU_MEMORY_MIB", "0") or 0),
            "memory_fraction": float(env.get("NANO_GPU_MEMORY_FRACTION", "0") or 0)}


def apply(device: int = 0) -> bool:
    frac = grant()["memory_fraction"]
    if frac <= 0:
        return False
    try:
        import torch
    except ImportError:
        return False
    if not torch.cuda.is_available():
        return False
    torch.cuda.set_per_process_memory_fraction(frac, device)
    return True
