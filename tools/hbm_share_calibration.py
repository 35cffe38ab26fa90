"""HBM-activity calibration per share (MI355X box): what amdgpu's mem_busy_percent reads while a
single CU-masked tenant runs alone on the GPU, for streaming (HBM copy) and compute-bound (bf16
MFMA burn) tenants at several shares of the CUs.

The learner in the ledger (Ledger::learn_stream_owners) decides whether the pod alone on a
device is streaming from that device's averaged activity. A 25 % streaming tenant alone moves
about half of the device's bandwidth (profiles/gpu_calibration.md), so a fixed full-chip
threshold would miss small streamers; this measures the activity curve the share-aware
threshold is built from (nanogpu.types.HBM_STREAMING_CURVE). Sampling: nanogpu.probe.calibrate
.mem_busy_while (a child process reads the counter every 10 ms; every sample of the window
counts, as in avg_over_time).

    python tools/hbm_share_calibration.py --out gpurun_out/hbm_share.json
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=8.0)
    ap.add_argument("--out", default="gpurun_out/hbm_share_calibration.json")
    ap.add_argument("--stream-shares", default="12.5,25,50,100")
    ap.add_argument("--mfma-shares", default="25,75,100")
    a = ap.parse_args(argv)

    import torch  # the HIP runtime first (nanogpu.native.probe loads after torch)

    assert torch.cuda.is_available(), "needs the GPU"
    from nanogpu.native import probe
    from nanogpu.probe import calibrate as C

    P = probe(required=True)
    f = C.mem_busy_file()
    if f is None:
        raise SystemExit("mem_busy_percent not exposed")
    runs = []
    for kind, shares in (("stream", a.stream_shares), ("mfma", a.mfma_shares)):
        for s in (float(x) for x in shares.split(",") if x):
            mask = C.cu_share_mask(s)
            runs.append((f"{kind} {s:g}% ({sum(bin(w).count('1') for w in mask)} CUs)", C.tenant_call(P, kind, mask)))
    res = {"file": str(f), "runs": C.mem_busy_while(f, runs, a.seconds)}
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(res, indent=1))
    print(json.dumps(res, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
