"""In-container side of a fractional MI355X grant (import it first, e.g. from sitecustomize).

The device plugin passes the grant through the environment (plugin.py):
  HSA_CU_MASK               spatial share, applied by ROCr itself when queues are created;
  GPU_MAX_HEAP_SIZE         the HBM budget in whole percents of the device, rounded up: the HIP
                            runtime reports that much memory as the device's total and refuses
                            any single allocation above it (it does not cap the sum);
  NANO_GPU_MEMORY_MIB       the exact HBM budget, applied here to the PyTorch caching allocator
  NANO_GPU_MEMORY_FRACTION  (the same budget as a fraction of the whole device, for readers that
                            do not see GPU_MAX_HEAP_SIZE). Cooperative: a process that bypasses
                            the allocator is capped only per allocation.
"""
from __future__ import annotations

import os


def grant() -> dict:
    env = os.environ
    return {"devices": env.get("NANO_GPU_DEVICES", ""), "percent": int(env.get("NANO_GPU_PERCENT", "0") or 0),
            "cu_mask": env.get("HSA_CU_MASK", ""), "memory_mib": int(env.get("NANO_GPU_MEMORY_MIB", "0") or 0),
            "memory_fraction": float(env.get("NANO_GPU_MEMORY_FRACTION", "0") or 0)}


def allocator_fraction(g: dict, reported_total_mib: float) -> float:
    """The PyTorch allocator's fraction for grant `g`: relative to the total the runtime
    reports, which GPU_MAX_HEAP_SIZE has already cut down to the rounded-up budget."""
    if g["memory_mib"] > 0 and reported_total_mib > 0:
        return min(1.0, g["memory_mib"] / reported_total_mib)
    return g["memory_fraction"]


def apply(device: int = 0) -> bool:
    g = grant()
    if g["memory_mib"] <= 0 and g["memory_fraction"] <= 0:
        return False
    try:
        import torch
    except ImportError:
        return False
    if not torch.cuda.is_available():
        return False
    total_mib = torch.cuda.get_device_properties(device).total_memory / (1 << 20)
    frac = allocator_fraction(g, total_mib)
    if frac <= 0:
        return False
    torch.cuda.set_per_process_memory_fraction(frac, device)
    return True
