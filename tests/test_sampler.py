"""Native CPU sampling profiler (native/src/sampler.cpp + nanogpu.obs.cpu_profile): the bench's
`--cpu-profile-out` substitute for perf, which the gpurun pool does not have."""
import threading
import time

from nanogpu import _native as N
from nanogpu.obs import cpu_profile


def test_sampler_attributes_cpu_to_threads_and_symbols():
    stop = threading.Event()

    def spin():   # a native busy loop on a second thread: the Go-1.16 sort permutation
        while not stop.is_set():
            N.go116_sort_perm(list(range(2000, 0, -1)))

    th = threading.Thread(target=spin)
    assert N.sampler_start(1000)
    assert not N.sampler_start(1000)          # one sampler per process
    th.start()
    t0 = time.process_time()
    while time.process_time() - t0 < 0.6:
        pass
    stop.set()
    th.join()
    samples = N.sampler_stop()
    assert N.sampler_stop() == []             # stopped
    assert len(samples) >= 20                 # the kernel's tick bounds the rate (~250 Hz a CPU)
    assert all(pc > 0 and tid > 0 for pc, _c, tid in samples)
    prof = cpu_profile(samples)
    assert prof["samples"] == len(samples)
    assert prof["main"]["samples"] > 0 and prof["other"]["samples"] > 0
    names = [n for g in ("main", "other") for n, _pct in prof[g]["top"]]
    assert any("python" in n or "libc" in n or "_native" in n for n in names), names
    assert abs(sum(p for _n, p in prof["main"]["top"]) - 100.0) < 1.0 or len(prof["main"]["top"]) == 25
