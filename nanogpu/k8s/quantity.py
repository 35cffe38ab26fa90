"""Kubernetes resource.Quantity parsing.

The reference reads limits with `Quantity.Value()` (pkg/utils/pod.go:94-100,
pkg/utils/node.go:8-14), which rounds UP to the nearest integer ("500m" -> 1,
"1.5" -> 2) [ext: k8s.io/apimachinery resource.Quantity semantics].
"""
from __future__ import annotations

import math
import re
from decimal import Decimal, InvalidOperation

_BINARY = {"Ki": 2 ** 10, "Mi": 2 ** 20, "Gi": 2 ** 30, "Ti": 2 ** 40, "Pi": 2 ** 50, "Ei": 2 ** 60}
_DECIMAL = {"n": Decimal("1e-9"), "u": Decimal("1e-6"), "m": Decimal("1e-3"), "": Decimal(1),
            "k": Decimal(10 ** 3), "M": Decimal(10 ** 6), "G": Decimal(10 ** 9),
            "T": Decimal(10 ** 12), "P": Decimal(10 ** 15), "E": Decimal(10 ** 18)}
_RE = re.compile(r"^([+-]?[0-9.]+)([eE][+-]?[0-9]+)?(Ki|Mi|Gi|Ti|Pi|Ei|n|u|m|k|M|G|T|P|E)?$")


class QuantityError(ValueError):
    pass


def parse_quantity(q) -> Decimal:
    """Exact value of a Quantity given as str/int/float."""
    if isinstance(q, bool):
        raise QuantityError(f"invalid quantity {q!r}")
    if isinstance(q, int):
        return Decimal(q)
    if isinstance(q, float):
        return Decimal(repr(q))
    if not isinstance(q, str):
        raise QuantityError(f"invalid quantity {q!r}")
    s = q.strip()
    m = _RE.match(s)
    if not m:
        raise QuantityError(f"invalid quantity {q!r}")
    num, exp, suffix = m.group(1), m.group(2), m.group(3) or ""
    try:
        v = Decimal(num)
        if exp:
            v = v * (Decimal(10) ** int(exp[1:]))
    except InvalidOperation as e:
        raise QuantityError(f"invalid quantity {q!r}") from e
    if suffix in _BINARY:
        return v * _BINARY[suffix]
    return v * _DECIMAL[suffix]


def quantity_value(q) -> int:
    """Quantity.Value(): integer value rounded up (away from zero for positives)."""
    v = parse_quantity(q)
    return int(math.ceil(v)) if v >= 0 else -int(math.ceil(-v))


def quantity_to_mib(q) -> int:
    """Memory-style quantity (bytes, 'Gi', ...) -> MiB, rounded up.

    `nano-gpu/gpu-memory` is expressed in MiB when given as a bare integer, so "32768"
    and "32Gi" both mean 32 GiB of HBM.
    """
    if isinstance(q, int) or (isinstance(q, str) and re.fullmatch(r"\s*[0-9]+\s*", q)):
        return int(q)
    v = parse_quantity(q)
    return int(math.ceil(v / (1 << 20)))
