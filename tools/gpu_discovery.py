"""One-shot hardware discovery on a real MI355X (run via gpurun).

Writes gpurun_out/discovery.json with: native topology reader output, HIP device props,
HBM bandwidth, CU-census (mask bit -> XCC/SE/CU), MFMA throughput vs CU mask; and copies
the KFD/DRM sysfs property files to gpurun_out/sysfs_capture/ (fixtures for CPU tests).
"""
from __future__ import annotations

import json
import os
import shutil
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
OUT = ROOT / "gpurun_out"
OUT.mkdir(exist_ok=True)


def capture_sysfs(dst: Path) -> list[str]:
    """Copies the sysfs facts into one tarball (gpurun merges a limited number of files)."""
    import tarfile
    import tempfile

    tmp = Path(tempfile.mkdtemp())
    files = _copy_sysfs(tmp)
    dst.parent.mkdir(parents=True, exist_ok=True)
    with tarfile.open(str(dst) + ".tar.gz", "w:gz") as tf:
        tf.add(str(tmp), arcname="root")
    shutil.rmtree(tmp, ignore_errors=True)
    return files


def _copy_sysfs(dst: Path) -> list[str]:
    copied = []
    kfd = Path("/sys/class/kfd/kfd/topology")
    for p in sorted(kfd.rglob("*")):
        try:
            if p.is_file() and p.stat().st_size < 65536:
                rel = p.relative_to("/")
                (dst / rel).parent.mkdir(parents=True, exist_ok=True)
                (dst / rel).write_text(p.read_text())
                copied.append(str(rel))
        except (OSError, UnicodeDecodeError):
            pass
    for card in sorted(Path("/sys/class/drm").glob("renderD*")):
        dev = card / "device"
        for name in ("current_compute_partition", "available_compute_partition", "current_memory_partition",
                     "available_memory_partition", "mem_info_vram_total", "numa_node", "unique_id",
                     "product_name", "vendor", "device"):
            f = dev / name
            try:
                txt = f.read_text()
            except OSError:
                continue
            rel = Path("sys/class/drm") / card.name / "device" / name
            (dst / rel).parent.mkdir(parents=True, exist_ok=True)
            (dst / rel).write_text(txt)
            copied.append(str(rel))
    return copied


def main() -> None:
    res: dict = {"time": time.time()}
    from nanogpu import _native as N

    host = json.loads(N.discover_topology("", True))
    res["topology"] = host
    print("topology gpus:", len(host["gpus"]), "links:", len(host["links"]), host.get("warnings"), flush=True)
    res["sysfs_files"] = len(capture_sysfs(OUT / "sysfs_capture"))

    from nanogpu import _probe as P

    res["device_count"] = P.device_count()
    res["props"] = P.device_props(0)
    print("props:", res["props"], flush=True)
    t = time.time()
    res["hbm_gbs"] = P.hbm_bandwidth(0, 1 << 30, 20)
    print(f"hbm copy: {res['hbm_gbs']:.1f} GB/s ({time.time() - t:.2f}s)", flush=True)

    cus = res["props"]["cus"]
    words = (cus + 31) // 32
    census = P.cu_census(0, [], 4096, 256)
    res["census_unmasked_distinct"] = len({c for c in census})
    res["census_unmasked_xcc"] = sorted({c[0] for c in census})
    # bit -> (xcc, hw_id) map: one launch per single-bit mask
    bitmap = {}
    for bit in range(cus):
        mask = [0] * words
        mask[bit // 32] = 1 << (bit % 32)
        recs = P.cu_census(0, mask, 64, 32)
        bitmap[bit] = sorted({r for r in recs})
    res["cu_bit_map"] = {str(k): v for k, v in bitmap.items()}
    print("bit->xcc (first 16):", [bitmap[b][0][0] if bitmap[b] else None for b in range(16)], flush=True)

    full = [0xFFFFFFFF] * words
    res["mfma_full"] = P.mfma_throughput(0, [], cus * 8, 4096)
    print("mfma unmasked:", res["mfma_full"], flush=True)
    scaling = {}
    for frac in (1, 2, 4, 8):
        n = cus // frac
        mask = [0] * words
        # first n bits
        for b in range(n):
            mask[b // 32] |= 1 << (b % 32)
        r = P.mfma_throughput(0, mask, cus * 8, 4096)
        scaling[str(n)] = r["tflops"]
        print(f"mfma with {n} CUs masked-in: {r['tflops']:.1f} TF/s", flush=True)
    res["mfma_mask_scaling"] = scaling
    (OUT / "discovery.json").write_text(json.dumps(res, indent=1))
    print("wrote", OUT / "discovery.json")


if __name__ == "__main__":
    main()
