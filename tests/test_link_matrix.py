"""Per-pair link calibration (nanogpu/probe/calibrate.py::link_matrix) as the bench runs it
with one rank per GPU: in round k every rank pulls from rank (r + k) % n, so each round is a
permutation over the links, and the rows are all-gathered. Rehearsed with gloo and a stand-in
probe whose "link rate" encodes the pair, so the assembled matrix can be checked exactly."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


class FakeProbe:
    def __init__(self, fail_pair=None, hang_pair=None):
        self.calls = []
        self.fail_pair = fail_pair
        self.hang_pair = hang_pair

    def peer_bandwidth(self, src, dst, nbytes, iters, deadline_s=30.0):
        import time

        self.calls.append((src, dst))
        if (src, dst) == self.fail_pair:
            raise RuntimeError("peer access denied")
        if (src, dst) == self.hang_pair:
            time.sleep(3600)          # a copy that never completes (and ignores its deadline)
        return {"gbs": 10.0 * src + dst + 1, "pull_gbs": 0.0, "dma_gbs": 0.0, "peer_access": True}


def _rank(rank, world, port, fail_pair, q, hang_pair=None):
    import time
    from datetime import timedelta

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from nanogpu.probe.calibrate import ProbeTimeout, link_matrix

    group = dist.new_group(backend="gloo", timeout=timedelta(seconds=60))
    fp = FakeProbe(fail_pair, hang_pair)
    t0 = time.monotonic()
    try:
        m = link_matrix(world, dist=dist, rank=rank, P=fp, group=group, pair_timeout_s=0.5)
        q.put((rank, "ok", m, fp.calls))
    except ProbeTimeout as e:
        q.put((rank, "timeout", (str(e), time.monotonic() - t0), fp.calls))
    except RuntimeError as e:
        q.put((rank, "error", str(e), fp.calls))
    dist.destroy_process_group()


def _run(world, fail_pair=None, hang_pair=None):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, world, port, fail_pair, q, hang_pair)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(60)
    return sorted(out)


@pytest.mark.parametrize("world", [2, 4])
def test_link_matrix_rounds_are_permutations_and_rows_gather(world):
    out = _run(world)
    for rank, status, m, calls in out:
        assert status == "ok"
        assert calls == [((rank + k) % world, rank) for k in range(1, world)]   # this rank's GPU pulls
        for a in range(world):
            for b in range(world):
                assert m[a][b] == (0.0 if a == b else 10.0 * a + b + 1)
    # round k: the (src, dst) pairs over all ranks form a permutation (each link direction once)
    for k in range(1, world):
        srcs = sorted(calls[k - 1][0] for _, _, _, calls in out)
        assert srcs == list(range(world))


def test_a_failed_pair_fails_every_rank_without_a_hang():
    out = _run(2, fail_pair=(1, 0))
    assert [status for _, status, _, _ in out] == ["error", "error"]


def test_a_hung_pair_times_out_on_every_rank():
    """One peer copy never completes: its rank gives up on it after the pair's time box and
    probes nothing more; every rank gets the same ProbeTimeout naming the pair, within a
    few time boxes (no rank blocks in a collective)."""
    out = _run(4, hang_pair=(1, 2))
    assert [status for _, status, _, _ in out] == ["timeout"] * 4, out
    for rank, _, (msg, took), calls in out:
        assert "1->2" in msg and took < 30
        if rank == 2:   # after the hung pull from GPU 1, GPU 2 pulls from no other peer
            assert calls == [(3, 2), (0, 2), (1, 2)][: calls.index((1, 2)) + 1]


def _busbw_rank(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from nanogpu.probe.calibrate import ring_busbw

    try:
        q.put((rank, "ok", ring_busbw(dist, "cpu", nbytes=4 << 20, iters=2)))
    except Exception as e:   # noqa: BLE001 - reported to the test
        q.put((rank, "error", f"{type(e).__name__}: {e}"))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_ring_busbw_runs_on_the_cpu_rehearsal(world):
    """The bench's N-GPU collective figure (RCCL all-reduce busBW) must not be able to abort a
    driver run: the same code runs over gloo on the CPU, and every rank reports one number."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_busbw_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
    assert all(st == "ok" for _, st, _ in out), out
    vals = {round(v, 6) for _, _, v in out}
    assert len(vals) == 1 and next(iter(vals)) > 0      # the max over ranks, the same everywhere


def _busbw_hang_rank(rank, world, port, q):
    import time
    from datetime import timedelta

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from nanogpu.probe import calibrate

    if rank == 1:   # this rank's ring never finishes
        calibrate.ring_busbw = lambda *a, **k: time.sleep(3600)
    agree = dist.new_group(backend="gloo", timeout=timedelta(seconds=60))
    t0 = time.monotonic()
    v, why = calibrate.ring_busbw_bounded(dist, "cpu", agree, timeout_s=2.0, nbytes=1 << 20, iters=1)
    q.put((rank, v, why, time.monotonic() - t0))
    dist.destroy_process_group()


def test_a_hung_ring_is_agreed_on_by_every_rank():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_busbw_hang_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(30)
        if p.is_alive():
            p.kill()
    for rank, v, why, took in out:
        assert v is None and why and took < 30, out
