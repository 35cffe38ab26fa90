"""Spatial sharing of one MI355X device: gpu-percent -> an XCD-symmetric CU mask.

The reference delegates "what does 20% of a GPU mean" to an NVIDIA device plugin
(reference README.md:9, 30-34; qgpu / MPS in its architecture diagram). On MI355X the
node agent makes a fractional grant *spatial*: the container's HSA queues get a CU mask
(ROCr `HSA_CU_MASK`, the same mechanism as `hipExtStreamCreateWithCUMask`) covering its
share of the device's compute units, disjoint from its neighbours' masks.

Mask-bit layout, measured on MI355X in SPX mode (tools/gpu_discovery.py, `cu_census`):
mask bit i enables a CU on XCD (i mod 8), and a dispatch round-robins workgroups over all
XCDs. A grant is therefore allocated in *units* of one CU per XCD (8 bits = 8 CUs =
3.125 % of a 256-CU device), which keeps every grant XCD-symmetric: each XCD (and its own
4 MiB L2) carries the same fraction of every tenant, and no tenant's workgroups queue
behind an XCD it owns alone. A CPX partition is one XCD, so its unit is one CU.

Sizing is floor(p/100 * units) (at least one unit), so any set of grants whose percents
sum to <= 100 fits; bf16 MFMA throughput scales linearly with the granted CUs
(tests/test_gpu.py::test_cu_mask_spatial_share_scales).
"""
from __future__ import annotations

from dataclasses import dataclass, field


@dataclass
class DeviceCUs:
    cus: int = 256
    xcds: int = 8
    used: dict[str, list[int]] = field(default_factory=dict)   # owner -> unit indices

    @property
    def unit(self) -> int:
        return max(1, self.xcds)

    @property
    def n_units(self) -> int:
        return self.cus // self.unit

    def units_for(self, percent: int) -> int:
        if percent >= 100:
            return self.n_units
        return max(1, (percent * self.n_units) // 100)

    def free_units(self) -> list[int]:
        taken = {u for us in self.used.values() for u in us}
        return [u for u in range(self.n_units) if u not in taken]

    def grant(self, owner: str, percent: int) -> list[int] | None:
        """Returns the CU bit indices granted to `owner` (idempotent), or None if full."""
        if owner in self.used:
            return self.bits(owner)
        need = self.units_for(percent)
        free = self.free_units()
        if len(free) < need:
            return None
        self.used[owner] = free[:need]
        return self.bits(owner)

    def restore(self, owner: str, bits: list[int]) -> None:
        """Re-registers a grant found in a pod annotation (agent restart)."""
        self.used[owner] = sorted({b // self.unit for b in bits})

    def release(self, owner: str) -> bool:
        return self.used.pop(owner, None) is not None

    def bits(self, owner: str) -> list[int]:
        return [u * self.unit + k for u in self.used[owner] for k in range(self.unit)]


def ranges(bits: list[int]) -> str:
    """[0,1,2,3,8,9] -> "0-3,8-9" (the HSA_CU_MASK CU-list syntax)."""
    out, bits = [], sorted(bits)
    i = 0
    while i < len(bits):
        j = i
        while j + 1 < len(bits) and bits[j + 1] == bits[j] + 1:
            j += 1
        out.append(f"{bits[i]}" if i == j else f"{bits[i]}-{bits[j]}")
        i = j + 1
    return ",".join(out)


def parse_ranges(text: str) -> list[int]:
    out = []
    for part in filter(None, (p.strip() for p in text.split(","))):
        a, _, b = part.partition("-")
        out.extend(range(int(a), int(b or a) + 1))
    return out


def hsa_cu_mask(device_index: int, bits: list[int]) -> str:
    """HSA_CU_MASK value for one visible device: "<index>:<cu-list>"."""
    return f"{device_index}:{ranges(bits)}"


def mask_words(bits: list[int], cus: int = 256) -> list[int]:
    """32-bit words for hipExtStreamCreateWithCUMask (the probe's masked streams)."""
    words = [0] * ((cus + 31) // 32)
    for b in bits:
        words[b // 32] |= 1 << (b % 32)
    return words
