"""List+watch informer and a de-duplicating async work queue.

Replaces client-go shared informers + workqueue (reference controller.go:89-136, 247-268).
The reference worker returns `false` after every successful item, so `wait.Until` sleeps a
second between items (controller.go:256-261, 185). These workers drain the
queue continuously and back off only on errors.
"""
from __future__ import annotations

import asyncio
import logging
import random
import time
from typing import Awaitable, Callable

from .client import ApiError

log = logging.getLogger(__name__)

Handler = Callable[[str, dict, dict | None], None]   # (event_type, obj, old_obj)


def _pod_key(o: dict) -> str:
    m = o.get("metadata") or {}
    return f"{m.get('namespace', '')}/{m.get('name', '')}"


def _node_key(o: dict) -> str:
    return (o.get("metadata") or {}).get("name", "")


def _rv(o: dict) -> str:
    return (o.get("metadata") or {}).get("resourceVersion", "")


class Informer:
    def __init__(self, api, resource: str, label_selector: str | None = None,
                 resync_s: float = 0.0, key=None, slim: bool = False, prefilter=None,
                 field_selector: str | None = None):
        self.api = api
        self.resource = resource               # "pods" | "nodes"
        self.label_selector = label_selector
        self.field_selector = field_selector   # pods: e.g. spec.nodeName=<node> (a node agent)
        self.resync_s = resync_s
        self.key = key or (_pod_key if resource == "pods" else _node_key)
        self.store: dict[str, dict] = {}
        self.handlers: list[Handler] = []
        # called after every LIST with (listed objects, time.monotonic() taken before the LIST
        # was sent): client-go's reflector Replace, for state kept outside this store
        self.relist_hooks: list[Callable[[list[dict], float], None]] = []
        self.synced = asyncio.Event()
        self.rv = ""
        self._task: asyncio.Task | None = None
        self.relists = 0      # LISTs (the first one included)
        self.rewatches = 0    # watches resumed from the last resourceVersion after a clean end
        self.expired = 0      # 410 Gone / expired resourceVersion answers (each forces a LIST)
        self.events = 0       # watch events handled
        # pods only: watch events decoded natively to the fields the controllers read (a
        # REST client that offers it; the in-process store shares its objects anyway)
        self.slim = slim and resource == "pods" and bool(getattr(api, "supports_slim_watch", False))
        # slim pods + a native ledger: the native filter does the pod controller's ledger-only
        # work (drops pending pods and bound pods the ledger holds, releases deletions of pods
        # never handed on) and passes on the rest; the store keeps only what it passed on
        self.watch_filter = None
        if self.slim and prefilter is not None:
            from ..native import core

            self.watch_filter = core().PodWatchFilter(prefilter)

    def add_handler(self, h: Handler) -> None:
        self.handlers.append(h)

    def add_relist_hook(self, h: Callable[[list[dict], float], None]) -> None:
        """`h(items, before)` runs after each LIST (awaited when it is a coroutine function; the
        watch resumes after it). The native watch filter keeps the pods this
        extender bound out of the store, so the store's diff below cannot see them vanish;
        the hook lets the ledger reconcile against the listed objects directly."""
        self.relist_hooks.append(h)

    def get(self, key: str) -> dict | None:
        return self.store.get(key)

    def list(self) -> list[dict]:
        return list(self.store.values())

    def _dispatch(self, etype: str, obj: dict, old: dict | None) -> None:
        for h in self.handlers:
            try:
                h(etype, obj, old)
            except Exception:  # a handler bug must not kill the informer
                log.exception("informer handler failed for %s %s", etype, self.key(obj))

    async def _list(self) -> None:
        before = time.monotonic()      # CLOCK_MONOTONIC, the ledger's clock (ledger.cpp mono_now)
        if self.resource == "pods":
            # slim: the LIST decoded natively to what the watch events carry too
            kw = {"slim": True} if self.slim else {}
            if self.field_selector:
                kw["field_selector"] = self.field_selector
            items, rv = await self.api.list_pods(label_selector=self.label_selector, **kw)
        else:
            items, rv = await self.api.list_nodes(label_selector=self.label_selector)
        fresh = {self.key(o): o for o in items}
        for k, old in list(self.store.items()):
            if k not in fresh:
                del self.store[k]
                self._dispatch("DELETED", old, None)
        for k, o in fresh.items():
            old = self.store.get(k)
            self.store[k] = o
            if old is not None and _rv(old) == _rv(o) and _rv(o):
                continue              # unchanged since we last saw it: nothing to hand on
            self._dispatch("MODIFIED" if old is not None else "ADDED", o, old)
        self.rv = rv
        self.relists += 1
        if getattr(self, "watch_filter", None) is not None:
            self.watch_filter.reset(list(self.store))   # everything listed is in the store now
        for h in self.relist_hooks:
            try:
                r = h(items, before)
                if asyncio.iscoroutine(r):   # a hook that moves its work off the loop
                    await r
            except Exception:  # a hook bug must not kill the informer
                log.exception("%s informer relist hook failed", self.resource)

    async def run(self) -> None:
        """client-go reflector semantics (/root/reference/go.mod:16, client-go v0.18 informers
        started at /root/reference/pkg/controller/controller.go:136): LIST once, then WATCH from
        the last resourceVersion seen. A watch that ends cleanly (the server's timeoutSeconds,
        a proxy closing the stream) is re-opened from that resourceVersion with no LIST. Only
        410 Gone / an ERROR event (the resourceVersion fell out of the server's watch cache)
        or a transport failure re-LISTs; the relist diff turns objects deleted while the watch
        was down into DELETED events."""
        backoff = 0.05
        need_list = True
        gone_in_a_row = 0
        while True:
            try:
                if need_list:
                    await self._list()
                    need_list = False
                    self.synced.set()
                t0, n0 = time.monotonic(), self.events
                await self._watch()
                gone_in_a_row = 0
                self.rewatches += 1          # clean end: resume from self.rv
                if self.events == n0 and time.monotonic() - t0 < 0.1:
                    # client-go's "very short watch": a server that closes every stream at once
                    # must not turn this loop into a busy one
                    await asyncio.sleep(backoff)
                    backoff = min(backoff * 2, 5.0)
                else:
                    backoff = 0.05
            except asyncio.CancelledError:
                raise
            except ApiError as e:
                need_list = True
                if e.status == 410:
                    self.expired += 1
                    gone_in_a_row += 1
                    if gone_in_a_row <= 3:
                        continue             # relist at once: the cache has moved past us
                else:
                    log.warning("%s informer: %s", self.resource, e)
                await asyncio.sleep(backoff)
                backoff = min(backoff * 2, 5.0)
            except Exception as e:  # transport failure: relist with backoff
                need_list = True
                log.warning("%s informer error: %s", self.resource, e)
                await asyncio.sleep(backoff + random.random() * backoff)
                backoff = min(backoff * 2, 5.0)

    async def _watch(self) -> None:
        # API objects that can (the in-process store, the REST client) deliver the stream in
        # batches: one loop wake-up per burst of events rather than one per event
        kw = {"field_selector": self.field_selector} if self.field_selector else {}
        if hasattr(self.api, "watch_batches"):
            if self.slim:
                kw.update(slim=True, watch_filter=self.watch_filter)
            stream = self.api.watch_batches(self.resource, self.rv, label_selector=self.label_selector, **kw)
        else:
            stream = _singletons(self.api.watch(self.resource, self.rv, label_selector=self.label_selector, **kw))
        try:
            await self._consume(stream)
        finally:
            # close the stream now, not when the generator is collected: a native watch thread
            # (client.py::_native_watch) would go on filtering into the relist that follows
            aclose = getattr(stream, "aclose", None)
            if aclose is not None:
                await aclose()

    async def _consume(self, stream) -> None:
        store, key, handlers = self.store, self.key, self.handlers
        pop, get = store.pop, store.get
        async for batch in stream:
            last = None
            self.events += len(batch)
            try:
                for ev in batch:
                    etype, obj = ev.get("type"), ev.get("object") or {}
                    if etype == "ERROR":
                        raise ApiError(int(obj.get("code", 500)), obj.get("message", "watch error"))
                    last = obj
                    if etype == "BOOKMARK":
                        continue
                    k = key(obj)
                    if etype == "DELETED":
                        old = pop(k, None)
                    else:
                        old = get(k)
                        store[k] = obj
                        if etype == "ADDED" and old is not None:
                            etype = "MODIFIED"
                        elif etype == "MODIFIED" and old is None:
                            etype = "ADDED"
                    if len(handlers) == 1:
                        try:
                            handlers[0](etype, obj, old)
                        except Exception:  # a handler bug must not kill the informer
                            log.exception("informer handler failed for %s %s", etype, k)
                    else:
                        self._dispatch(etype, obj, old)
            finally:
                # resume point: the last event handled (events arrive in resourceVersion order)
                if last is not None:
                    self.rv = (last.get("metadata") or {}).get("resourceVersion", self.rv)

    def start(self) -> asyncio.Task:
        self._task = asyncio.ensure_future(self.run())
        return self._task

    async def stop(self) -> None:
        if self._task:
            self._task.cancel()
            try:
                await self._task
            except (asyncio.CancelledError, Exception):
                pass


async def _singletons(events):
    async for ev in events:
        yield (ev,)


class WorkQueue:
    """Keyed queue: a key is processed by at most one worker at a time and queued once."""

    def __init__(self, name: str, max_retries: int = 5, base_backoff: float = 0.01, max_backoff: float = 5.0):
        self.name = name
        self.q: asyncio.Queue[str] = asyncio.Queue()
        self.queued: set[str] = set()
        self.processing: set[str] = set()
        self.dirty: set[str] = set()
        self.retries: dict[str, int] = {}
        self.max_retries = max_retries
        self.base_backoff = base_backoff
        self.max_backoff = max_backoff
        self.processed = 0
        self.dropped = 0

    def add(self, key: str) -> None:
        if key in self.processing:
            self.dirty.add(key)
            return
        if key in self.queued:
            return
        self.queued.add(key)
        self.q.put_nowait(key)

    def depth(self) -> int:
        return self.q.qsize()

    async def _process(self, key: str, fn: Callable[[str], Awaitable[None]]) -> None:
        self.queued.discard(key)
        self.processing.add(key)
        try:
            await fn(key)
            self.retries.pop(key, None)
            self.processed += 1
        except asyncio.CancelledError:
            raise
        except Exception as e:
            n = self.retries.get(key, 0) + 1
            if n > self.max_retries:
                log.error("%s: dropping %s after %d retries: %s", self.name, key, n - 1, e)
                self.retries.pop(key, None)
                self.dropped += 1
            else:
                self.retries[key] = n
                delay = min(self.base_backoff * 2 ** (n - 1), self.max_backoff)
                asyncio.get_running_loop().call_later(delay, self.add, key)
        finally:
            self.processing.discard(key)
            if key in self.dirty:
                self.dirty.discard(key)
                self.add(key)

    async def worker(self, fn: Callable[[str], Awaitable[None]]) -> None:
        while True:
            key = await self.q.get()
            await self._process(key, fn)

    async def drain(self, timeout: float = 10.0) -> bool:
        loop = asyncio.get_running_loop()
        end = loop.time() + timeout
        while (self.q.qsize() or self.processing) and loop.time() < end:
            await asyncio.sleep(0.002)
        return not (self.q.qsize() or self.processing)
