"""Minimal async Kubernetes REST client (pods, nodes, bindings, events, watch).

Replaces client-go v0.18 (reference go.mod:16) for the calls the reference makes:
List pods by label/field selector (dealer.go:58-60, 279-282), Get pod (bind.go:62, 68),
Update pod (dealer.go:177, 184) -> here a JSON merge-patch of annotations/labels only,
which cannot hit the optimistic-lock path the reference mishandles (D1), Create
pods/binding (dealer.go:191-197), informers (list+watch) and the events sink.
"""
from __future__ import annotations

import asyncio
import base64
import json
import logging
import os
import ssl
import tempfile
import time
import urllib.parse
from dataclasses import dataclass
from typing import Any, AsyncIterator

import aiohttp

log = logging.getLogger(__name__)

SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"


class ApiError(Exception):
    def __init__(self, status: int, message: str, reason: str = "", retry_after: float | None = None):
        super().__init__(f"{status} {reason}: {message}")
        self.status = status
        self.reason = reason
        self.message = message
        self.retry_after = retry_after   # seconds, from a 429's Retry-After header

    @property
    def throttled(self) -> bool:
        """kube-apiserver's max-in-flight admission refused the request (nothing was done)."""
        return self.status == 429

    @property
    def not_found(self) -> bool:
        return self.status == 404

    @property
    def conflict(self) -> bool:
        return self.status == 409


def _retry_after(headers) -> float | None:
    v = headers.get("Retry-After") if headers is not None else None
    try:
        return float(v) if v is not None else None
    except ValueError:
        return None


@dataclass
class KubeConfig:
    server: str
    token: str | None = None
    ca_file: str | None = None
    cert_file: str | None = None
    key_file: str | None = None
    insecure: bool = False
    token_file: str | None = None      # re-read while running (projected tokens rotate)

    @classmethod
    def in_cluster(cls) -> "KubeConfig":
        host, port = os.environ.get("KUBERNETES_SERVICE_HOST"), os.environ.get("KUBERNETES_SERVICE_PORT")
        if not host or not port:
            raise RuntimeError("not running in a cluster (KUBERNETES_SERVICE_HOST unset)")
        token_file = os.path.join(SA_DIR, "token")
        with open(token_file) as f:
            token = f.read().strip()
        if ":" in host:
            host = f"[{host}]"
        return cls(server=f"https://{host}:{port}", token=token, ca_file=os.path.join(SA_DIR, "ca.crt"),
                   token_file=token_file)

    @classmethod
    def from_kubeconfig(cls, path: str, context: str | None = None) -> "KubeConfig":
        import yaml

        with open(path) as f:
            cfg = yaml.safe_load(f) or {}
        ctx_name = context or cfg.get("current-context")
        ctx = next((c["context"] for c in cfg.get("contexts", []) if c.get("name") == ctx_name), None)
        if ctx is None:
            raise RuntimeError(f"kubeconfig {path}: context {ctx_name!r} not found")
        cluster = next(c["cluster"] for c in cfg.get("clusters", []) if c.get("name") == ctx["cluster"])
        user = next((u.get("user") or {} for u in cfg.get("users", []) if u.get("name") == ctx.get("user")), {})

        def materialise(data_key: str, file_key: str, src: dict) -> str | None:
            if src.get(file_key):
                return src[file_key]
            if src.get(data_key):
                fd, p = tempfile.mkstemp(prefix="nanogpu-kc-")
                with os.fdopen(fd, "wb") as f:
                    f.write(base64.b64decode(src[data_key]))
                return p
            return None

        token_file = user.get("tokenFile")
        token = user.get("token")
        if not token and token_file:
            with open(token_file) as f:
                token = f.read().strip()
        return cls(server=cluster["server"].rstrip("/"), token=token, token_file=token_file,
                   ca_file=materialise("certificate-authority-data", "certificate-authority", cluster),
                   cert_file=materialise("client-certificate-data", "client-certificate", user),
                   key_file=materialise("client-key-data", "client-key", user),
                   insecure=bool(cluster.get("insecure-skip-tls-verify")))

    @classmethod
    def auto(cls, kubeconfig: str | None = None, server: str | None = None) -> "KubeConfig":
        """KUBECONFIG env / path first, then in-cluster (reference cmd/main.go:42-61)."""
        if server:
            return cls(server=server.rstrip("/"))
        path = kubeconfig or os.environ.get("KUBECONFIG")
        if path:
            return cls.from_kubeconfig(path)
        return cls.in_cluster()

    def ssl_context(self) -> ssl.SSLContext | bool:
        if not self.server.startswith("https"):
            return False
        ctx = ssl.create_default_context(cafile=self.ca_file) if self.ca_file else ssl.create_default_context()
        if self.insecure:
            ctx.check_hostname = False
            ctx.verify_mode = ssl.CERT_NONE
        if self.cert_file and self.key_file:
            ctx.load_cert_chain(self.cert_file, self.key_file)
        return ctx


async def _ndjson_batches(chunks, decode=None) -> AsyncIterator[list[dict]]:
    """Newline-delimited JSON from a byte stream: the complete lines of each chunk as a list
    (a partial last line waits for the next chunk). `decode(bytes) -> list` replaces
    json.loads per line (the native slim pod decoder)."""
    tail = b""
    async for chunk in chunks:
        data = tail + chunk if tail else chunk
        cut = data.rfind(b"\n")
        if cut < 0:
            tail = data
            continue
        tail = data[cut + 1:]
        if decode is not None:
            batch = decode(data[:cut])
        else:
            batch = [json.loads(line) for line in data[:cut].split(b"\n") if line.strip()]
        if batch:
            yield batch


class KubeClient:
    """Async client; one keep-alive connection pool per process.

    Bearer tokens from a file (the in-cluster service-account token, a kubeconfig
    `tokenFile`) are re-read when the file changes, checked at most every
    `token_check_s`, and at once after a 401: kubelet rotates projected tokens while the
    extender keeps running (client-go reloads them the same way)."""

    supports_slim_watch = True   # watch_batches(slim=True): native slim pod decoding

    def __init__(self, config: KubeConfig, timeout_s: float = 30.0, pool: int = 64, token_check_s: float = 60.0,
                 native_watch: bool = True):
        self.config = config
        # a filtered pod watch (watch_batches with a watch_filter) is read by a native thread
        # (nanogpu._native.PodWatchStream) rather than by aiohttp on the event loop
        u = urllib.parse.urlsplit(config.server)
        self.native_watch = native_watch and u.scheme in ("http", "https") and bool(u.hostname)
        self._timeout = aiohttp.ClientTimeout(total=timeout_s)
        self._pool = pool
        self._session: aiohttp.ClientSession | None = None
        self.calls = 0
        self.token_check_s = token_check_s
        self._token = config.token
        self._token_mtime = self._mtime()
        self._token_checked = time.monotonic()

    def _mtime(self) -> float:
        try:
            return os.stat(self.config.token_file).st_mtime if self.config.token_file else 0.0
        except OSError:
            return 0.0

    def _auth(self, force: bool = False) -> dict | None:
        """Authorization header for the next request (re-reading a rotated token file)."""
        if self.config.token_file:
            now = time.monotonic()
            if force or now - self._token_checked >= self.token_check_s:
                self._token_checked = now
                m = self._mtime()
                if force or m != self._token_mtime:
                    try:
                        with open(self.config.token_file) as f:
                            self._token = f.read().strip() or self._token
                        self._token_mtime = m
                    except OSError:
                        pass
        return {"Authorization": f"Bearer {self._token}"} if self._token else None

    async def _s(self) -> aiohttp.ClientSession:
        if self._session is None or self._session.closed:
            headers = {"Accept": "application/json", "User-Agent": "nano-gpu-scheduler-amd/0.1"}
            self._session = aiohttp.ClientSession(
                headers=headers, timeout=self._timeout,
                connector=aiohttp.TCPConnector(limit=self._pool, ssl=self.config.ssl_context()),
                json_serialize=lambda o: json.dumps(o, separators=(",", ":")))
        return self._session

    async def close(self) -> None:
        if self._session is not None:
            await self._session.close()
            self._session = None

    async def request(self, method: str, path: str, body: Any = None, params: dict | None = None,
                      content_type: str = "application/json") -> Any:
        s = await self._s()
        url = self.config.server + path
        data = None if body is None else json.dumps(body, separators=(",", ":"))
        for attempt in (0, 1):
            self.calls += 1
            headers = dict(self._auth(force=attempt == 1) or {})
            if data is not None:
                headers["Content-Type"] = content_type
            async with s.request(method, url, data=data, params=params, headers=headers or None) as r:
                text = await r.text()
                status = r.status
                ra = _retry_after(r.headers) if status == 429 else None
            if status == 401 and attempt == 0 and self.config.token_file:
                continue                      # the token may have rotated under us: re-read once
            break
        if status >= 400:
            try:
                st = json.loads(text)
                raise ApiError(status, st.get("message", text), st.get("reason", ""), ra)
            except (ValueError, AttributeError):
                raise ApiError(status, text, "", ra) from None
        return json.loads(text) if text else None

    # --------------------------------------------------------------------- pods
    async def get_pod(self, ns: str, name: str) -> dict:
        return await self.request("GET", f"/api/v1/namespaces/{ns}/pods/{name}")

    async def patch_pod(self, ns: str, name: str, patch: dict) -> dict:
        return await self.request("PATCH", f"/api/v1/namespaces/{ns}/pods/{name}", patch,
                                  content_type="application/merge-patch+json")

    async def bind_pod(self, ns: str, name: str, uid: str, node: str, annotations: dict | None = None) -> None:
        """pods/binding; `annotations` land on the pod atomically with spec.nodeName."""
        md = {"name": name, "namespace": ns, "uid": uid}
        if annotations:
            md["annotations"] = annotations
        body = {"apiVersion": "v1", "kind": "Binding", "metadata": md,
                "target": {"apiVersion": "v1", "kind": "Node", "name": node}}
        await self.request("POST", f"/api/v1/namespaces/{ns}/pods/{name}/binding", body)

    async def create_pod(self, pod: dict) -> dict:
        ns = (pod.get("metadata") or {}).get("namespace", "default")
        return await self.request("POST", f"/api/v1/namespaces/{ns}/pods", pod)

    async def delete_pod(self, ns: str, name: str) -> None:
        await self.request("DELETE", f"/api/v1/namespaces/{ns}/pods/{name}")

    async def request_bytes(self, method: str, path: str, params: dict | None = None) -> bytes:
        """`request` without decoding: the body as bytes (raises ApiError as `request` does)."""
        s = await self._s()
        for attempt in (0, 1):
            self.calls += 1
            headers = dict(self._auth(force=attempt == 1) or {})
            async with s.request(method, self.config.server + path, params=params, headers=headers or None) as r:
                body = await r.read()
                status = r.status
                ra = _retry_after(r.headers) if status == 429 else None
            if status == 401 and attempt == 0 and self.config.token_file:
                continue
            break
        if status >= 400:
            text = body.decode("utf-8", "replace")
            try:
                st = json.loads(text)
                raise ApiError(status, st.get("message", text), st.get("reason", ""), ra)
            except (ValueError, AttributeError):
                raise ApiError(status, text, "", ra) from None
        return body

    async def list_pods(self, label_selector: str | None = None, field_selector: str | None = None,
                        namespace: str | None = None, slim: bool = False, page: int = 500) -> tuple[list[dict], str]:
        """All pods matching the selectors, read `page` at a time (`limit` / `continue`, as
        client-go's pager: a 100k-pod LIST is never one body in memory); a continue token that
        expired meanwhile (410) restarts as one unpaged LIST. `slim`: each page decoded natively
        down to what the pod informer reads (nanogpu._native.decode_pod_list), the rest of every
        pod never becomes a Python object."""
        params = {}
        if label_selector:
            params["labelSelector"] = label_selector
        if field_selector:
            params["fieldSelector"] = field_selector
        path = f"/api/v1/namespaces/{namespace}/pods" if namespace else "/api/v1/pods"
        decode = None
        if slim:
            from ..native import core

            decode = core().decode_pod_list
        items: list[dict] = []
        rv, cont = "", ""
        try:
            while True:
                q = dict(params, limit=str(page)) if page > 0 else dict(params)
                if cont:
                    q["continue"] = cont
                if decode is not None:
                    got, rv, cont = decode(await self.request_bytes("GET", path, params=q))
                else:
                    r = await self.request("GET", path, params=q or None)
                    got = r.get("items") or []
                    md = r.get("metadata") or {}
                    rv, cont = md.get("resourceVersion", ""), md.get("continue", "")
                items.extend(got)
                if not cont or page <= 0:
                    return items, rv
        except ApiError as e:
            if e.status != 410 or page <= 0:
                raise
            return await self.list_pods(label_selector, field_selector, namespace, slim=slim, page=0)

    # --------------------------------------------------------------------- nodes
    async def get_node(self, name: str) -> dict:
        return await self.request("GET", f"/api/v1/nodes/{name}")

    async def list_nodes(self, label_selector: str | None = None) -> tuple[list[dict], str]:
        r = await self.request("GET", "/api/v1/nodes",
                               params={"labelSelector": label_selector} if label_selector else None)
        return r.get("items") or [], (r.get("metadata") or {}).get("resourceVersion", "")

    async def patch_node(self, name: str, patch: dict) -> dict:
        return await self.request("PATCH", f"/api/v1/nodes/{name}", patch,
                                  content_type="application/merge-patch+json")

    async def patch_node_status(self, name: str, patch: dict) -> dict:
        return await self.request("PATCH", f"/api/v1/nodes/{name}/status", patch,
                                  content_type="application/merge-patch+json")

    # --------------------------------------------------------------------- leases
    async def get_lease(self, ns: str, name: str) -> dict:
        return await self.request("GET", f"/apis/coordination.k8s.io/v1/namespaces/{ns}/leases/{name}")

    async def create_lease(self, ns: str, lease: dict) -> dict:
        return await self.request("POST", f"/apis/coordination.k8s.io/v1/namespaces/{ns}/leases", lease)

    async def update_lease(self, ns: str, name: str, lease: dict) -> dict:
        return await self.request("PUT", f"/apis/coordination.k8s.io/v1/namespaces/{ns}/leases/{name}", lease)

    # --------------------------------------------------------------------- events
    async def create_event(self, ns: str, involved: dict, reason: str, message: str,
                           etype: str = "Warning") -> None:
        import time
        import uuid

        ts = time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())
        body = {"apiVersion": "v1", "kind": "Event",
                "metadata": {"name": f"{involved.get('name', 'obj')}.{uuid.uuid4().hex[:10]}", "namespace": ns},
                "involvedObject": involved, "reason": reason, "message": message, "type": etype,
                "source": {"component": "nano-gpu-scheduler"}, "firstTimestamp": ts, "lastTimestamp": ts,
                "count": 1}
        try:
            await self.request("POST", f"/api/v1/namespaces/{ns}/events", body)
        except (ApiError, aiohttp.ClientError, asyncio.TimeoutError) as e:
            log.debug("event not recorded: %s", e)

    # --------------------------------------------------------------------- watch
    async def watch(self, resource: str, resource_version: str, timeout_s: int = 300,
                    label_selector: str | None = None, field_selector: str | None = None) -> AsyncIterator[dict]:
        """Streams watch events ({type, object}) for `pods` or `nodes` cluster-wide."""
        s = await self._s()
        params = {"watch": "1", "resourceVersion": resource_version, "timeoutSeconds": str(timeout_s),
                  "allowWatchBookmarks": "true"}
        if label_selector:
            params["labelSelector"] = label_selector
        if field_selector:
            params["fieldSelector"] = field_selector
        url = f"{self.config.server}/api/v1/{resource}?{urllib.parse.urlencode(params)}"
        async with s.get(url, timeout=aiohttp.ClientTimeout(total=None, sock_read=timeout_s + 30),
                         headers=self._auth()) as r:
            if r.status >= 400:
                raise ApiError(r.status, await r.text())
            async for batch in _ndjson_batches(r.content.iter_any()):
                for ev in batch:
                    yield ev

    async def _native_watch(self, path: str, watch_filter, read_timeout_s: int) -> AsyncIterator[list[dict]]:
        """The filtered pod watch on a native thread (native/src/podwatch.cpp): the stream is
        read, split and filtered off the event loop, which wakes only for the events the filter
        keeps. Errors as in the aiohttp path: ApiError for an HTTP error answer, a transport
        failure as an exception the informer relists on, a clean end as the end of the stream."""
        from ..native import core

        u = urllib.parse.urlsplit(self.config.server)
        tls = u.scheme == "https"
        hdr = self._auth() or {}
        token = hdr.get("Authorization", "")[len("Bearer "):]
        c = self.config
        st = core().PodWatchStream(u.hostname, u.port or (443 if tls else 80), tls, token, c.ca_file or "",
                                   c.cert_file or "", c.key_file or "", bool(c.insecure),
                                   u.path.rstrip("/") + path, watch_filter, read_timeout_s)
        loop = asyncio.get_running_loop()
        ready = asyncio.Event()
        fd = st.notify_fd()
        loop.add_reader(fd, ready.set)
        try:
            while True:
                await ready.wait()
                ready.clear()
                events, state, status, message = st.take()
                if events:
                    yield events
                if state == 1:
                    return
                if state == 2:
                    raise ApiError(status, message)
                if state == 3:
                    raise ConnectionError(f"pod watch: {message}")
        finally:
            loop.remove_reader(fd)
            st.stop()   # shuts the socket down and joins the thread (no blocking read left)

    async def watch_batches(self, resource: str, resource_version: str, timeout_s: int = 300,
                            label_selector: str | None = None, slim: bool = False,
                            watch_filter=None, field_selector: str | None = None) -> AsyncIterator[list[dict]]:
        """`watch`, one list per network read: every complete event line that arrived together.
        slim (pods): each Pod decoded natively down to what the pod informer reads
        (nanogpu._native.decode_pod_watch) instead of json.loads of the whole object; a
        `watch_filter` (nanogpu._native.PodWatchFilter) also does the pod controller's
        ledger-only work natively and passes on only the rest."""
        decode = None
        if slim and resource == "pods":
            from ..native import core

            decode = watch_filter.decode if watch_filter is not None else core().decode_pod_watch
        params = {"watch": "1", "resourceVersion": resource_version, "timeoutSeconds": str(timeout_s),
                  "allowWatchBookmarks": "true"}
        if label_selector:
            params["labelSelector"] = label_selector
        if field_selector:
            params["fieldSelector"] = field_selector
        if decode is not None and watch_filter is not None and self.native_watch:
            async for batch in self._native_watch(f"/api/v1/{resource}?{urllib.parse.urlencode(params)}",
                                                  watch_filter, timeout_s + 30):
                yield batch
            return
        s = await self._s()
        url = f"{self.config.server}/api/v1/{resource}?{urllib.parse.urlencode(params)}"
        async with s.get(url, timeout=aiohttp.ClientTimeout(total=None, sock_read=timeout_s + 30),
                         headers=self._auth()) as r:
            if r.status >= 400:
                raise ApiError(r.status, await r.text())
            async for batch in _ndjson_batches(r.content.iter_any(), decode):
                yield batch
