"""Bulk create / delete of 1000-pod bursts on the native API server with one watcher
(bench.py's shared API server path, without the ranks). Prints per-burst server times."""
import json
import os
import socket
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from nanogpu.native import core  # noqa: E402

srv = core().ApiServer("127.0.0.1", 0, 4, 1 << 16)
got = [0]


def reader(s):
    while True:
        b = s.recv(1 << 20)
        if not b:
            return
        got[0] += len(b)


s = socket.create_connection(("127.0.0.1", srv.port))
s.sendall(b"GET /api/v1/pods?watch=true&resourceVersion=0 HTTP/1.1\r\nHost: x\r\n\r\n")
threading.Thread(target=reader, args=(s,), daemon=True).start()
time.sleep(0.2)
tc, td = [], []
for step in range(int(sys.argv[1]) if len(sys.argv) > 1 else 20):
    texts = [json.dumps(p, separators=(",", ":")) for p in bench.burst(0, 1, 1000, step, 7)]
    keys = [(m.get("namespace", "default"), m["name"]) for m in (json.loads(t)["metadata"] for t in texts)]
    t = time.perf_counter()
    srv.create_pods(texts)
    tc.append(time.perf_counter() - t)
    t = time.perf_counter()
    srv.delete_pods(keys)
    td.append(time.perf_counter() - t)
tc.sort()
td.sort()
print(json.dumps({"bulk_threads": os.environ.get("NANOGPU_APISERVER_BULK_THREADS", "4"),
                  "create_ms_p50": round(1e3 * tc[len(tc) // 2], 3), "delete_ms_p50": round(1e3 * td[len(td) // 2], 3),
                  "create_ms_min": round(1e3 * tc[0], 3), "delete_ms_min": round(1e3 * td[0], 3)}))
srv.stop()
