"""Node calibration on real MI355X hardware: facts the scheduler's node model needs.

* local_gpu_facts()  — native KFD/amdsmi reader + HIP device props (CUs, HBM bytes, gfx,
  partition modes, NUMA) for the GPU this process owns;
* hbm_bandwidth()    — streaming-copy GB/s from the HIP probe kernel;
* cu_mask_isolation()— bf16 MFMA TFLOP/s on CU-masked streams (the agent's spatial share);
* link_matrix()      — per-pair xGMI rates (GB/s, one direction) from the peer-pull probe:
  what the topology scorer weights GPU groups with. Single process: every visible pair in
  turn. One rank per GPU: rank r pulls from (r + k) % n in round k, so each round is a
  permutation and every link direction carries exactly one transfer; rows are all-gathered.
* reader_link_gbs()  — the per-link rate KFD publishes (io_link max_bandwidth), when the
  peers themselves are hidden from this process (a 1-GPU container still sees its links).
* ring_busbw()       — RCCL all-reduce bus bandwidth across the job's ranks (torch.distributed
  backend "nccl" = RCCL on ROCm). An aggregate collective figure: on a full xGMI mesh RCCL
  drives several links at once, so it is reported as such and never as a per-link rate.
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
    P = probe(required=True, build=True)
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


def reader_link_gbs(host: dict) -> float:
    """Slowest xGMI link of the first visible GPU as KFD reports it, GB/s (0: none)."""
    gpus = host.get("gpus") or []
    return float(gpus[0].get("xgmi_min_bw_mbs", 0)) / 1000.0 if gpus else 0.0


class ProbeTimeout(RuntimeError):
    """A calibration step that did not finish in its time box (a wedged link, peer or RCCL
    ring); the node model falls back to the rates KFD publishes."""


def bounded(fn, timeout_s: float):
    """Runs `fn()` on a daemon thread for at most `timeout_s`: ("ok", value), ("error", exc)
    or ("timeout", None). A call stuck inside the HIP runtime or RCCL is abandoned, not
    joined, so the rank reaches its next collective and the job agrees on the outcome."""
    import threading

    box: dict = {}

    def run():
        try:
            box["v"] = fn()
        except BaseException as e:   # noqa: BLE001 - reported to the caller
            box["e"] = e

    th = threading.Thread(target=run, daemon=True, name="ngpu-probe")
    th.start()
    th.join(timeout_s)
    if th.is_alive():
        return "timeout", None
    if "e" in box:
        return ("timeout" if isinstance(box["e"], TimeoutError) else "error"), box["e"]
    return "ok", box["v"]


_TIMEOUT, _ERROR = -2.0, -1.0


def link_matrix(n: int, nbytes: int = 64 << 20, iters: int = 3, dist=None, rank: int = 0,
                P=None, group=None, pair_timeout_s: float = 30.0) -> list[list[float]]:
    """n x n per-direction GB/s, m[src][dst], from the peer-pull probe (0 on the diagonal).
    `P`: the probe module (tests pass a stand-in). Every pair is time-boxed (`bounded`, and the
    probe's own event deadline): after a timeout a rank probes nothing more on its GPU. With
    `dist`, rounds are kept in step and the rows exchanged over `group` (a gloo group with a
    timeout: CPU-side, so a wedged GPU stream cannot hold it); every rank then holds the same
    matrix and raises the same ProbeTimeout / RuntimeError, so they all fall back together."""
    P = P or probe(required=True)
    m = [[0.0] * n for _ in range(n)]

    def pair(src: int, dst: int) -> float:
        kind, v = bounded(lambda: P.peer_bandwidth(src, dst, nbytes, iters, pair_timeout_s), pair_timeout_s + 5.0)
        return v["gbs"] if kind == "ok" else _TIMEOUT if kind == "timeout" else _ERROR

    if dist is None:
        wedged = False
        for dst in range(n):
            for src in range(n):
                if src != dst:
                    m[src][dst] = _TIMEOUT if wedged else pair(src, dst)
                    wedged = wedged or m[src][dst] == _TIMEOUT
    else:
        import torch

        row = [0.0] * n                      # this rank's GPU as the destination
        wedged = False
        for k in range(1, n):
            src = (rank + k) % n
            dist.barrier(group=group)
            row[src] = _TIMEOUT if wedged else pair(src, rank)
            wedged = wedged or row[src] == _TIMEOUT
        t = torch.tensor(row, dtype=torch.float64)
        rows = [torch.zeros_like(t) for _ in range(n)]
        dist.all_gather(rows, t, group=group)
        for dst, r in enumerate(rows):
            for src, v in enumerate(r.tolist()):
                m[src][dst] = v
    late = [f"{s}->{d}" for s in range(n) for d in range(n) if m[s][d] == _TIMEOUT]
    if late:
        raise ProbeTimeout(f"peer copy timed out ({pair_timeout_s:g} s per pair): {', '.join(late[:8])}"
                           + (f" and {len(late) - 8} more" if len(late) > 8 else ""))
    if any(v < 0 for r in m for v in r):  # every rank sees the same gathered matrix
        raise RuntimeError("peer_bandwidth failed on some pair")
    return m


def agree(dist, ok: bool, group=None) -> bool:
    """True on every rank iff `ok` on every rank (one MIN all-reduce over `group`)."""
    import torch

    t = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(t.item())


def ring_busbw(dist, device, nbytes: int = 256 << 20, iters: int = 5, group=None) -> float:
    """RCCL all-reduce bus bandwidth (GB/s) over all ranks of the job: busBW = 2(n-1)/n x
    bytes / t. A collective aggregate (several xGMI links at once on a full mesh), not a
    per-link rate. `group`: the communicator to measure on (the bench gives it one of its own,
    so a ring that wedges cannot hold the job's default group)."""
    import torch

    n = dist.get_world_size()
    dev = torch.device(device)
    # gloo (the CPU rehearsal) reduces float32; RCCL moves bf16, as a training job would
    buf = torch.ones(nbytes // 2, dtype=torch.bfloat16 if dev.type == "cuda" else torch.float32, device=dev)
    nbytes = buf.numel() * buf.element_size()

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    dist.all_reduce(buf, group=group)   # warm-up (communicator setup)
    sync()
    t0 = time.perf_counter()
    for _ in range(iters):
        dist.all_reduce(buf, group=group)
    sync()
    dt = (time.perf_counter() - t0) / iters
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return 2.0 * (n - 1) / n * nbytes / float(t.item()) / 1e9


def ring_busbw_bounded(dist, device, agree_group, timeout_s: float = 60.0, **kw) -> tuple[float | None, str]:
    """`ring_busbw` in a time box on a communicator of its own, then one agreement over the
    CPU `agree_group`: (GB/s, "") when every rank finished, else (None, why) on every rank."""
    import torch

    if torch.device(device).type == "cuda":
        torch.cuda.set_device(torch.device(device))
    from datetime import timedelta

    ring = dist.new_group(backend="nccl" if torch.device(device).type == "cuda" else "gloo",
                          timeout=timedelta(seconds=max(1.0, timeout_s)))

    def run():
        if torch.device(device).type == "cuda":
            torch.cuda.set_device(torch.device(device))   # this thread's current device
        return ring_busbw(dist, device, group=ring, **kw)

    kind, v = bounded(run, timeout_s)
    ok = agree(dist, kind == "ok", group=agree_group)
    if ok:
        return v, ""
    return None, ("RCCL all-reduce timed out" if kind == "timeout" else
                  f"RCCL all-reduce failed: {type(v).__name__}: {v}" if kind == "error" else
                  "RCCL all-reduce failed or timed out on another rank")


# --------------------------------------------------------------------------- HBM activity
_SAMPLER = r"""
import json, sys, time
f = open(sys.argv[1]); end = time.monotonic() + float(sys.argv[2]); out = []
while time.monotonic() < end:
    f.seek(0); out.append((time.monotonic(), int(f.read() or 0))); time.sleep(0.01)
print(json.dumps(out))
"""


def mem_busy_file(host: dict | None = None):
    """amdgpu's mem_busy_percent of the GPU this process sees first (None: not exposed)."""
    from pathlib import Path

    host = host if host is not None else json.loads(core().discover_topology("", True))
    for g in host.get("gpus") or []:
        p = Path(f"/sys/class/drm/renderD{int(g['render_minor'])}/device/mem_busy_percent")
        if p.exists():
            return p
    return next(iter(sorted(Path("/sys/class/drm").glob("renderD*/device/mem_busy_percent"))), None)


def mem_busy_files(host: dict | None = None) -> dict:
    """Physical GPU index (topology GpuSpec.index: the reader's `parent`) -> its amdgpu
    mem_busy_percent file, for the GPUs that expose one."""
    from pathlib import Path

    host = host if host is not None else json.loads(core().discover_topology("", True))
    out = {}
    for k, g in enumerate(host.get("gpus") or []):
        p = Path(f"/sys/class/drm/renderD{int(g['render_minor'])}/device/mem_busy_percent")
        if p.exists():
            out.setdefault(int(g.get("parent", k)), p)
    return out


def hbm_busy_calibration(P, device: int, busy_file, shares=(25, 100), seconds: float = 3.0) -> list:
    """This GPU's own mem_busy_percent scale (topology GpuSpec.hbm_busy_cal): the probe's HBM
    stream alone on `device` under a CU mask of each share for `seconds`, with every 10 ms
    sample of `busy_file` averaged. The same kernels at the same GB/s read 54.4 / 30.1 % on one
    box and 28.7 / 20.7 % on another, so the classifier (types.HBM_HOT_THRESHOLD, the learner's
    curve) compares a device's readings with its own scale (telemetry.store.normalize_hbm_activity)
    instead of one box's constants. [[share %, mean mem_busy %], ...]; [] when the counter
    never moved (not exposed, or an idle-reading device)."""
    if busy_file is None:
        return []
    runs = [(f"stream{s}", tenant_call(P, "stream", cu_share_mask(s), device)) for s in shares]
    res = mem_busy_while(busy_file, runs, seconds=seconds)
    cal = [[float(s), float(r["mean_all"] or 0.0)] for s, r in zip(shares, res)]
    return cal if all(b > 0 for _, b in cal) else []


def cu_share_mask(share_pct: float, cus: int = 256, xcds: int = 8) -> list[int]:
    """Mask words of the node agent's grant for a `share_pct` % tenant (nanogpu.agent.cumask)."""
    from ..agent import cumask

    if share_pct >= 100:
        return cumask.mask_words(list(range(cus)), cus)
    d = cumask.DeviceCUs(cus, xcds)
    return cumask.mask_words(d.grant("t", int(round(share_pct))), cus)


def tenant_call(P, kind: str, mask: list[int], device: int = 0, seconds: float = 1.0):
    """A callable that runs about `seconds` of one CU-masked tenant: "stream" (HBM copy, returns
    GB/s) or "mfma" (bf16 burn, returns TFLOP/s). Each probe launch is bounded, so long runs
    call it back to back."""
    n_cus = sum(bin(w).count("1") for w in mask)
    if kind == "stream":
        t = time.perf_counter()
        P.hbm_colocated(device, [mask], 1 << 30, 4)
        iters = max(4, min(1000, int(seconds / max((time.perf_counter() - t) / 4, 1e-5))))
        return lambda: P.hbm_colocated(device, [mask], 1 << 30, iters)[0]
    blocks = max(8, n_cus * 8)
    t = time.perf_counter()
    P.mfma_throughput(device, mask, blocks, 4096)
    iters = max(4096, min(1 << 22, int(4096 * seconds / max(time.perf_counter() - t, 1e-6))))
    return lambda: P.mfma_throughput(device, mask, blocks, iters)["tflops"]


def mem_busy_while(busy_file, runs: list, seconds: float = 8.0, ramp_s: float = 0.3) -> list[dict]:
    """Runs each (label, callable) of `runs` back to back for `seconds` while a child process
    samples `busy_file` every 10 ms (a probe call may hold the GIL). Per run: the mean of ALL
    samples in its window (what avg_over_time over scrapes converges to), the max, the mean of
    the non-zero samples, and means at scrape-like spacing (1 s, 5 s); plus the call's rate."""
    import subprocess
    import sys

    total = len(runs) * (seconds + 2.0) + 5.0
    sampler = subprocess.Popen([sys.executable, "-c", _SAMPLER, str(busy_file), str(total)],
                               stdout=subprocess.PIPE, text=True)
    time.sleep(0.3)
    windows = []
    try:
        for label, call in runs:
            got = []
            t0 = time.monotonic()
            while time.monotonic() - t0 < seconds:
                got.append(call())
            windows.append((label, t0 + ramp_s, time.monotonic(), sum(got) / len(got), len(got)))
            time.sleep(0.5)
    finally:
        out, _ = sampler.communicate(timeout=total + 30)
    samples = json.loads(out)
    res = []
    for label, t0, t1, rate, calls in windows:
        win = [(t, v) for t, v in samples if t0 <= t <= t1]
        vals = [v for _, v in win]

        def spaced(step: float):
            picked, nxt = [], t0 + step / 2
            for t, v in win:
                if t >= nxt:
                    picked.append(v)
                    nxt += step
            return round(sum(picked) / len(picked), 1) if picked else None

        nz = [v for v in vals if v]
        res.append({"label": label, "seconds": round(t1 - t0, 2), "rate": round(rate, 1), "calls": calls,
                    "n": len(vals), "mean_all": round(sum(vals) / len(vals), 1) if vals else None,
                    "max": max(vals) if vals else None,
                    "mean_nonzero": round(sum(nz) / len(nz), 1) if nz else 0.0,
                    "mean_1s": spaced(1.0), "mean_5s": spaced(5.0)})
    return res
