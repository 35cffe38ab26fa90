"""Watch streams: NDJSON framing across network reads, batched delivery from the in-process
store (history replay, label selectors, drop = end of stream)."""
import asyncio
import json

from nanogpu.k8s import podutil as pu
from nanogpu.k8s.client import _ndjson_batches
from nanogpu.k8s.fake_apiserver import FakeKubeStore


def test_ndjson_batches_reassemble_lines_split_across_chunks():
    evs = [{"type": "ADDED", "object": {"metadata": {"name": f"p{i}", "resourceVersion": str(i)}}} for i in range(5)]
    raw = b"".join(json.dumps(e).encode() + b"\n" for e in evs)
    cuts = [0, 7, 8, 60, 61, len(raw) - 3, len(raw)]

    async def chunks():
        for a, b in zip(cuts, cuts[1:]):
            yield raw[a:b]

    async def main():
        return [b async for b in _ndjson_batches(chunks())]

    batches = asyncio.run(main())
    assert [e for b in batches for e in b] == evs
    assert all(batches)                       # no empty batches


def test_store_watch_batches_replay_selector_and_drop():
    store = FakeKubeStore()

    async def main():
        store.create_pod(pu.make_pod("old", [("c", 10)]))
        got = []

        async def consume():
            async for batch in store.watch_batches("pods", "0", label_selector="app=x"):
                got.append([pu.meta(e["object"])["name"] for e in batch])

        t = asyncio.ensure_future(consume())
        await asyncio.sleep(0)
        for i in range(3):                    # a burst: arrives as one batch
            p = pu.make_pod(f"x{i}", [("c", 10)])
            p["metadata"]["labels"] = {"app": "x"}
            store.create_pod(p)
        await asyncio.sleep(0)
        store.drop_watches()
        await asyncio.wait_for(t, 2.0)
        return got

    got = asyncio.run(main())
    assert got == [["x0", "x1", "x2"]]        # "old" replayed but filtered by the selector
