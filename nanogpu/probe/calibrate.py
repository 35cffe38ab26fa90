"""Node calibration on real MI355X hardware: facts the scheduler's node model needs.

* local_gpu_facts()  — native KFD/amdsmi reader + HIP device props (CUs, HBM bytes, gfx,
  partition modes, NUMA) for the GPU this process owns;
* hbm_bandwidth()    — streaming-copy GB/s from the HIP probe kernel;
* cu_mask_isolation()— bf16 MFMA TFLOP/s on CU-masked streams (the agent's spatial share);
* link_matrix()      — per-pair xGMI bandwidth measured with RCCL (torch.distributed,
  backend "nccl" = RCCL on ROCm) between the ranks of one node; feeds the topology scorer.
"""
from __future__ import annotations

import json
import time

from ..native import core, probe


def local_gpu_facts(device: int = 0, use_probe: bool = True) -> dict:
    N = core()
    host = json.loads(N.discover_topology("", True))
    facts: dict = {"host": host}
    P = probe(required=False) if use_probe else None
    if P is not None:
        try:
            facts["props"] = P.device_props(device)
        except RuntimeError as e:  # no GPU visible
            facts["props_error"] = str(e)
    return facts


def hbm_bandwidth(device: int = 0, nbytes: int = 1 << 30, iters: int = 10) -> float:
    P = probe(required=True)
    return P.hbm_bandwidth(device, nbytes, iters)


def interleaved_mask(n_cus: int, total_cus: int = 256, n_xcd: int = 8) -> list[int]:
    """CU-mask words for the first `n_cus` CUs, spread evenly over the XCDs.

    Measured on MI355X (tools/gpu_discovery.py): in SPX mode mask bit i feeds XCD i % 8,
    and a dispatch round-robins its workgroups over all XCDs, so a share must be
    XCD-symmetric; the granularity is one CU per XCD (8 CUs = 3.125%)."""
    words = [0] * ((total_cus + 31) // 32)
    for b in range(min(n_cus, total_cus)):
        words[b // 32] |= 1 << (b % 32)
    return words


def cu_mask_isolation(device: int = 0, fractions=(1, 2, 4, 8), iters: int = 2048) -> dict:
    P = probe(required=True)
    props = P.device_props(device)
    cus = props["cus"]
    out = {}
    for f in fractions:
        n = cus // f
        r = P.mfma_throughput(device, interleaved_mask(n, cus), cus * 8, iters)
        out[n] = r["tflops"]
    return out


def link_matrix(dist, device, nbytes: int = 64 << 20, iters: int = 5) -> list[list[float]]:
    """Pairwise RCCL bandwidth (GB/s) between all ranks, via 2-rank sub-groups.

    Every pair of MI355X GPUs in a node is one xGMI hop, so the matrix is expected to be
    near-uniform; measuring it catches degraded links and PCIe-only pairs."""
    import torch

    world, rank = dist.get_world_size(), dist.get_rank()
    bw = [[0.0] * world for _ in range(world)]
    buf = torch.ones(nbytes // 2, dtype=torch.bfloat16, device=device)
    for a in range(world):
        for b in range(a + 1, world):
            g = dist.new_group([a, b])
            if rank in (a, b):
                dist.all_reduce(buf, group=g)  # warm-up
                torch.cuda.synchronize(device)
                t0 = time.perf_counter()
                for _ in range(iters):
                    dist.all_reduce(buf, group=g)
                torch.cuda.synchronize(device)
                dt = (time.perf_counter() - t0) / iters
                # 2-rank ring all-reduce moves 2*(n-1)/n * bytes = bytes per rank
                bw[a][b] = bw[b][a] = nbytes / dt / 1e9
            dist.barrier()
    t = torch.tensor(bw, dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.cpu().tolist()
