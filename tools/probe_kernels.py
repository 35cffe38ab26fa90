"""Runs every HIP probe kernel once on plain streams (no CU-mask streams): the target for
`rocprofv3 --kernel-trace --stats` (CU-masked stream creation is left out because it is
not needed for per-kernel timing). Prints one JSON line with the measured rates."""
from __future__ import annotations

import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main() -> None:
    from nanogpu.native import probe

    P = probe(required=True)
    out = {"props": P.device_props(0)}
    out["copy_ok"] = P.copy_check(0, 1 << 24)
    out["hbm_gbs"] = {str(mb): round(P.hbm_bandwidth(0, mb << 20, 20), 1) for mb in (256, 1024, 4096)}
    out["mfma"] = P.mfma_throughput(0, [], 2048, 4096)
    a = [float((i % 7) - 3) for i in range(32 * 16)]
    b = [float((i % 5) - 2) for i in range(16 * 32)]
    out["gemm_tile_c00"] = P.gemm_tile(a, b)[0]
    out["census_xcc"] = sorted({x for x, _ in P.cu_census(0, [], 2048, 16)})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
