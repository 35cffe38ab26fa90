"""Load telemetry store: per (node, metric, card) latest utilisation in [0, 1].

Reference: pkg/dealer/nodeusage.go (string values + "Asia/Shanghai" wall-clock strings,
re-parsed and tzdata-loaded on every filter: nodeusage.go:82-111, stats.go:30-55, D13).
Here values are floats with monotonic timestamps, and the derived per-device load
(`usage = Σ_metrics ceil(10u)/10`, RemainLoad = 2 - int(usage), allocate.go:173-195) is
pushed into the native ledger when it changes, not recomputed inside the hot path.
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass

from .. import types as T


@dataclass
class Sample:
    value: float
    t: float


class TelemetryStore:
    def __init__(self):
        self.data: dict[tuple[str, str, int], Sample] = {}

    def update(self, node: str, metric: str, card: int, value: float, t: float | None = None) -> None:
        self.data[(node, metric, card)] = Sample(float(value), time.monotonic() if t is None else t)

    def get(self, node: str, metric: str, card: int, active_s: float, now: float | None = None
            ) -> tuple[bool, float, str | None]:
        """(exists, value, error) like Dealer.GetUsage (nodeusage.go:82-111)."""
        s = self.data.get((node, metric, card))
        if s is None:
            return False, 0.0, None
        now = time.monotonic() if now is None else now
        if now > s.t + active_s:
            return True, 0.0, f"{metric} not in update period"
        if not (0.0 <= s.value <= 1.0) or math.isnan(s.value):
            return True, 0.0, f"{metric} usage < 0 || usage > 1"
        return True, s.value, None

    def device_usage(self, node: str, card: int, periods: list[tuple[str, float]], now: float | None = None
                     ) -> float:
        """Σ over policy metrics of ceil(10u)/10 for fresh, valid samples (allocate.go:173-195)."""
        total = 0.0
        for metric, active_s in periods:
            if active_s <= 0:
                continue
            exists, v, err = self.get(node, metric, card, active_s, now)
            if not exists or err:
                continue
            total += math.ceil(10 * v) / 10
        return total

    def hbm_activity(self, node: str, card: int, active_s: float, now: float | None = None) -> float:
        """Fresh, valid HBM-activity sample in [0, 1]; 0.0 when stale, missing or invalid."""
        if active_s <= 0:
            return 0.0
        exists, v, err = self.get(node, T.GPU_HBM_ACTIVITY_METRIC, card, active_s, now)
        return v if exists and err is None else 0.0

    def hbm_hot(self, node: str, card: int, active_s: float, threshold: float, now: float | None = None
                ) -> bool:
        """Fresh, valid HBM-activity sample at or above `threshold` (types.GPU_HBM_ACTIVITY_METRIC)."""
        if active_s <= 0:
            return False
        exists, v, err = self.get(node, T.GPU_HBM_ACTIVITY_METRIC, card, active_s, now)
        return exists and err is None and v >= threshold

    def nodes(self) -> set[str]:
        return {k[0] for k in self.data}


def normalize_hbm_activity(v: float, cal: list | None) -> float:
    """A device's HBM activity (0..1, amdgpu mem_busy_percent / 100) on the scale of the
    calibration box the classifier's constants come from (types.HBM_STREAMING_CURVE,
    HBM_HOT_THRESHOLD). `cal` is that device's own curve, [[CU share %, mem_busy %], ...] of a
    lone streaming probe (GpuSpec.hbm_busy_cal): the reading is mapped piecewise-linearly through
    (0, 0) and each calibrated point onto the reference curve at the same share, so a quarter-GPU
    streamer reads as one on every box (one box: 20.7 % where the calibration box read 30.1 %).
    The reference (prometheus.go:70-76, allocate.go:173-195) likewise normalises load values
    before bucketing them. No calibration: the reading as it is."""
    pts = sorted((float(s), float(b)) for s, b in (cal or []) if b > 0)
    if not pts or v <= 0:
        return max(0.0, v)
    ref = T.HBM_STREAMING_CURVE

    def ref_at(share: float) -> float:
        if share <= ref[0][0]:
            return ref[0][1] * share / ref[0][0]
        for (s0, b0), (s1, b1) in zip(ref, ref[1:]):
            if share <= s1:
                return b0 + (b1 - b0) * (share - s0) / (s1 - s0)
        return ref[-1][1]

    xs = [0.0] + [b for _, b in pts]
    ys = [0.0] + [ref_at(s) for s, _ in pts]
    x = 100.0 * v
    for k in range(1, len(xs)):
        if x <= xs[k] or k == len(xs) - 1:
            x0, x1, y0, y1 = xs[k - 1], xs[k], ys[k - 1], ys[k]
            y = y0 + (y1 - y0) * (x - x0) / (x1 - x0) if x1 > x0 else y1
            return max(0.0, min(1.0, y / 100.0))
    return max(0.0, min(1.0, v))

