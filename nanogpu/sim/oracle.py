"""Reference-behaviour oracle: the reference's placement algebra in plain Python.

No Go toolchain is available, so parity is pinned against this independent executable
specification of SURVEY.md Appendix B (reference pkg/dealer/rater.go:59-163,
allocate.go:92-131, 225-247), including Go 1.16 `sort.Sort` ordering. The C++ `compat`
mode is diffed against it by property tests (tests/test_parity.py), and the frag/quality
benches replay the same pod stream through it to report "reference" numbers.
"""
from __future__ import annotations

from dataclasses import dataclass


# ------------------------------------------------------------------ Go 1.16 sort.Sort
def go116_sort(data: list, key) -> None:
    """In-place, with Go 1.16's exact swap sequence (less(i, j) := key(d[i]) < key(d[j]))."""

    def less(i, j):
        return key(data[i]) < key(data[j])

    def swap(i, j):
        data[i], data[j] = data[j], data[i]

    def insertion(a, b):
        for i in range(a + 1, b):
            j = i
            while j > a and less(j, j - 1):
                swap(j, j - 1)
                j -= 1

    def sift_down(lo, hi, first):
        root = lo
        while True:
            child = 2 * root + 1
            if child >= hi:
                return
            if child + 1 < hi and less(first + child, first + child + 1):
                child += 1
            if not less(first + root, first + child):
                return
            swap(first + root, first + child)
            root = child

    def heap_sort(a, b):
        first, hi = a, b - a
        for i in range((hi - 1) // 2, -1, -1):
            sift_down(i, hi, first)
        for i in range(hi - 1, -1, -1):
            swap(first, first + i)
            sift_down(0, i, first)

    def median3(m1, m0, m2):
        if less(m1, m0):
            swap(m1, m0)
        if less(m2, m1):
            swap(m2, m1)
            if less(m1, m0):
                swap(m1, m0)

    def do_pivot(lo, hi):
        m = (lo + hi) >> 1
        if hi - lo > 40:
            s = (hi - lo) // 8
            median3(lo, lo + s, lo + 2 * s)
            median3(m, m - s, m + s)
            median3(hi - 1, hi - 1 - s, hi - 1 - 2 * s)
        median3(lo, m, hi - 1)
        pivot = lo
        a, c = lo + 1, hi - 1
        while a < c and less(a, pivot):
            a += 1
        b = a
        while True:
            while b < c and not less(pivot, b):
                b += 1
            while b < c and less(pivot, c - 1):
                c -= 1
            if b >= c:
                break
            swap(b, c - 1)
            b += 1
            c -= 1
        protect = hi - c < 5
        if not protect and hi - c < (hi - lo) // 4:
            dups = 0
            if not less(pivot, hi - 1):
                swap(c, hi - 1)
                c += 1
                dups += 1
            if not less(b - 1, pivot):
                b -= 1
                dups += 1
            if not less(m, pivot):
                swap(m, b - 1)
                b -= 1
                dups += 1
            protect = dups > 1
        if protect:
            while True:
                while a < b and not less(b - 1, pivot):
                    b -= 1
                while a < b and less(a, pivot):
                    a += 1
                if a >= b:
                    break
                swap(a, b - 1)
                a += 1
                b -= 1
        swap(pivot, b - 1)
        return b - 1, c

    def quick(a, b, depth):
        while b - a > 12:
            if depth == 0:
                heap_sort(a, b)
                return
            depth -= 1
            mlo, mhi = do_pivot(a, b)
            if mlo - a < b - mhi:
                quick(a, mlo, depth)
                a = mhi
            else:
                quick(mhi, b, depth)
                b = mlo
        if b - a > 1:
            for i in range(a + 6, b):
                if less(i, i - 6):
                    swap(i, i - 6)
            insertion(a, b)

    n = len(data)
    depth, i = 0, n
    while i > 0:
        depth += 1
        i >>= 1
    quick(0, n, depth * 2)


# ------------------------------------------------------------------ GPUResource algebra
@dataclass
class G:
    percent: int
    total: int = 100
    remain_load: int = 0
    index: int = 0


def rate_binpack(gpus: list[G], load_usage: float = 0.0) -> int:
    if not gpus:
        raise ZeroDivisionError("integer divide by zero")  # reference panics (D6)
    s = sum(g.total for g in gpus)
    used = sum(g.total - g.percent for g in gpus)
    usage = float(used) / float(s)
    load_int = int(load_usage) // len(gpus)
    return int(usage * 100) + load_int * 50 - len(gpus)


def rate_spread(gpus: list[G], load_usage: float = 0.0) -> int:
    if not gpus:
        raise ZeroDivisionError("integer divide by zero")
    avail = sum(g.percent for g in gpus)
    free = sum(1 for g in gpus if g.percent == g.total)
    load_int = int(load_usage) // len(gpus)
    return 100 * free + avail // 10 - len(gpus) - load_int


def choose(gpus: list[G], demand: list[int], spread: bool) -> list[int] | None:
    """Binpack.Choose / Spread.Choose; None when the reference returns an error."""
    sg = [G(g.percent, g.total, g.remain_load, i) for i, g in enumerate(gpus)]
    sd = [G(p, 0, 0, i) for i, p in enumerate(demand)]
    go116_sort(sd, key=lambda x: x.percent + x.remain_load * 50)
    indexes: list[int] = []
    for j in range(len(sd) - 1, -1, -1):
        if sd[j].percent == 0:
            indexes.append(-1)
            continue
        go116_sort(sg, key=lambda x: x.percent + x.remain_load * 50)
        order = range(len(sg) - 1, -1, -1) if spread else range(len(sg))
        for i in order:
            if sg[i].percent >= sd[j].percent:
                indexes.append(sg[i].index)
                sg[i].percent -= sd[j].percent
                break
    if len(indexes) != len(demand):
        return None
    result = [0] * len(demand)
    for j in range(len(demand) - 1, -1, -1):
        result[sd[j].index] = indexes[len(demand) - 1 - j]
    return result


def first_fit(gpus: list[G], demand: list[int]) -> list[int] | None:
    free = [g.percent for g in gpus]
    out = []
    for p in demand:
        if p == 0:
            out.append(-1)
            continue
        for j, f in enumerate(free):
            if f >= p:
                out.append(j)
                free[j] -= p
                break
    return out if len(out) == len(demand) else None


class OracleCluster:
    """Whole-cluster reference model (for replaying pod streams: frag and throughput parity)."""

    def __init__(self, nodes: dict[str, int], policy: str = "binpack"):
        self.policy = policy
        self.nodes = {n: [G(100, 100, 0, i) for i in range(c)] for n, c in nodes.items()}
        self.pods: dict[str, tuple[str, list[int], list[int]]] = {}

    def score(self, node: str) -> int:
        g = self.nodes[node]
        return rate_spread(g) if self.policy == "spread" else rate_binpack(g)

    def fits(self, node: str, demand: list[int]) -> list[int] | None:
        g = self.nodes[node]
        if not g:
            return None
        return choose(g, demand, self.policy == "spread")

    def schedule(self, uid: str, demand: list[int], candidates: list[str]) -> str | None:
        best, host = None, None
        for n in candidates:
            plan = self.fits(n, demand)
            if plan is None:
                continue
            s = self.score(n)
            if best is None or s > best:
                best, host = s, n
        if host is None:
            return None
        plan = self.fits(host, demand)
        for p, i in zip(demand, plan):
            if i >= 0:
                self.nodes[host][i].percent -= p
        self.pods[uid] = (host, demand, plan)
        return host

    def release(self, uid: str) -> None:
        host, demand, plan = self.pods.pop(uid)
        for p, i in zip(demand, plan):
            if i >= 0:
                self.nodes[host][i].percent += p

    def frag(self) -> dict:
        free = sum(g.percent for gs in self.nodes.values() for g in gs)
        partial = sum(g.percent for gs in self.nodes.values() for g in gs if 0 < g.percent < g.total)
        return {"pct_free_total": free, "pct_free_partial": partial,
                "frag_pct": 100.0 * partial / free if free else 0.0}
