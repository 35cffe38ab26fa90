"""CPU placement (nanogpu.affinity) on a synthetic sysfs tree shaped like the MI355X host:
2 sockets, L3 domains of physical cores with SMT siblings offset by the core count."""
from pathlib import Path

from nanogpu import affinity as A


def make_tree(root: Path, sockets=2, doms_per_socket=3, cores_per_dom=4) -> set[int]:
    ncores = sockets * doms_per_socket * cores_per_dom
    for core in range(ncores):
        dom = core // cores_per_dom
        node = dom // doms_per_socket
        l3 = [c for c in range(ncores) if c // cores_per_dom == dom]
        l3_all = l3 + [c + ncores for c in l3]
        for cpu in (core, core + ncores):           # SMT siblings
            base = root / f"cpu{cpu}"
            (base / "topology").mkdir(parents=True)
            (base / "topology" / "thread_siblings_list").write_text(f"{core},{core + ncores}\n")
            idx = base / "cache" / "index3"
            idx.mkdir(parents=True)
            (idx / "level").write_text("3\n")
            (idx / "shared_cpu_list").write_text(f"{l3_all[0]}-{l3_all[len(l3) - 1]},{l3_all[len(l3)]}-{l3_all[-1]}\n")
            (base / f"node{node}").mkdir()
    return set(range(2 * ncores))


def test_domains_are_physical_cores_per_l3(tmp_path):
    allowed = make_tree(tmp_path)
    doms = A.l3_domains(allowed, root=tmp_path)
    assert doms == [[0, 1, 2, 3], [4, 5, 6, 7], [8, 9, 10, 11], [12, 13, 14, 15], [16, 17, 18, 19],
                    [20, 21, 22, 23]]
    assert A.numa_of_cpu(13, root=tmp_path) == 1
    # a restricted cpuset keeps only what it allows (here: no SMT siblings at all)
    assert A.l3_domains({8, 9, 30}, root=tmp_path) == [[8, 9]]


def test_ranks_of_a_node_get_distinct_domains_on_their_gpu_numa(tmp_path, monkeypatch):
    allowed = make_tree(tmp_path)
    monkeypatch.setattr(A, "SYS_CPU", tmp_path)
    monkeypatch.setattr(A.os, "sched_getaffinity", lambda pid: allowed)
    real_l3, real_numa = A.l3_domains, A.numa_of_cpu
    monkeypatch.setattr(A, "l3_domains", lambda allowed=None, root=tmp_path: real_l3(allowed, root))
    monkeypatch.setattr(A, "numa_of_cpu", lambda cpu, root=tmp_path: real_numa(cpu, root))
    gpu_numa = [0, 0, 1, 1]                          # 4 ranks, two GPUs per socket
    picks = [A.pick_cpus(gpu_numa[r], r, gpu_numa) for r in range(4)]
    # CPU 0's domain is skipped; each rank stays on its GPU's socket; no domain is shared
    assert picks == [[4, 5, 6, 7], [8, 9, 10, 11], [12, 13, 14, 15], [16, 17, 18, 19]]


def test_single_rank_takes_the_least_busy_domain(tmp_path, monkeypatch):
    allowed = make_tree(tmp_path)
    real_l3, real_numa = A.l3_domains, A.numa_of_cpu
    monkeypatch.setattr(A.os, "sched_getaffinity", lambda pid: allowed)
    monkeypatch.setattr(A, "l3_domains", lambda allowed=None, root=tmp_path: real_l3(allowed, root))
    monkeypatch.setattr(A, "numa_of_cpu", lambda cpu, root=tmp_path: real_numa(cpu, root))
    busy = {c: 0.9 for c in range(24)}
    busy.update({c: 0.1 for c in (8, 9, 10, 11)})
    monkeypatch.setattr(A, "_busy", lambda cpus, w: {c: busy.get(c, 0.0) for c in cpus})
    assert A.pick_cpus(0) == [8, 9, 10, 11]
    assert A.pick_cpus(1) in ([12, 13, 14, 15], [16, 17, 18, 19], [20, 21, 22, 23])


def test_bench_api_server_keeps_off_every_ranks_domain(tmp_path, monkeypatch):
    """The shared API server starts before the ranks are busy, so it must avoid their
    domains by construction, not by load: the least busy free domain, rank 0's socket on a tie."""
    allowed = make_tree(tmp_path)
    real_l3, real_numa = A.l3_domains, A.numa_of_cpu
    monkeypatch.setattr(A.os, "sched_getaffinity", lambda pid: allowed)
    monkeypatch.setattr(A, "l3_domains", lambda allowed=None, root=tmp_path: real_l3(allowed, root))
    monkeypatch.setattr(A, "numa_of_cpu", lambda cpu, root=tmp_path: real_numa(cpu, root))
    monkeypatch.setattr(A, "_busy", lambda cpus, w: {c: 0.0 for c in cpus})   # all idle
    gpu_numa = [0, 0, 1, 1]
    taken = [c for r in range(4) for c in A.pick_cpus(gpu_numa[r], r, gpu_numa)]
    assert A.pick_cpus_avoiding(taken, near=0) == [20, 21, 22, 23]   # socket 0 has no free domain but CPU 0's
    assert A.pick_cpus_avoiding(taken[:4], near=0) == [8, 9, 10, 11]
    assert A.pick_cpus_avoiding(taken[:4], near=1) == [12, 13, 14, 15]


def test_bench_api_server_stays_on_rank0s_socket_unless_it_is_busy(tmp_path, monkeypatch):
    """A near-socket domain that is a little busier (a shared host) still beats an idle domain
    on the far socket: every bind and watch event would cross the socket otherwise. Only a
    near domain at least half busy loses to a quieter far one."""
    allowed = make_tree(tmp_path)
    real_l3, real_numa = A.l3_domains, A.numa_of_cpu
    monkeypatch.setattr(A.os, "sched_getaffinity", lambda pid: allowed)
    monkeypatch.setattr(A, "l3_domains", lambda allowed=None, root=tmp_path: real_l3(allowed, root))
    monkeypatch.setattr(A, "numa_of_cpu", lambda cpu, root=tmp_path: real_numa(cpu, root))
    busy = {c: 0.0 for c in range(24)}
    busy.update({c: 0.2 for c in (8, 9, 10, 11)})          # socket 0's free domain: lightly used
    monkeypatch.setattr(A, "_busy", lambda cpus, w: {c: busy.get(c, 0.0) for c in cpus})
    taken = A.pick_cpus(0, 0, [0])                          # rank 0 on socket 0
    assert A.numa_of_cpu(taken[0]) == 0
    assert A.pick_cpus_avoiding(taken, near=0) == [8, 9, 10, 11]
    busy.update({c: 0.7 for c in (8, 9, 10, 11)})           # now mostly busy: go far
    assert A.numa_of_cpu(A.pick_cpus_avoiding(taken, near=0)[0]) == 1


def test_a_domain_whose_smt_siblings_are_busy_loses(tmp_path, monkeypatch):
    """Two idle domains on the GPU's socket; another tenant keeps the SMT siblings of one of
    them busy: the rank takes the other (the siblings' load counts with the cores')."""
    allowed = make_tree(tmp_path)
    monkeypatch.setattr(A, "SYS_CPU", tmp_path)
    real_l3, real_numa = A.l3_domains, A.numa_of_cpu
    monkeypatch.setattr(A.os, "sched_getaffinity", lambda pid: allowed)
    monkeypatch.setattr(A, "l3_domains", lambda allowed=None, root=tmp_path: real_l3(allowed, root))
    monkeypatch.setattr(A, "numa_of_cpu", lambda cpu, root=tmp_path: real_numa(cpu, root))
    busy = {c: 0.0 for c in range(48)}
    busy.update({c + 24: 0.8 for c in (4, 5, 6, 7)})       # siblings of domain [4..7]
    monkeypatch.setattr(A, "_busy", lambda cpus, w: {c: busy.get(c, 0.0) for c in cpus})
    assert A.smt_siblings([4, 5]) == [28, 29]
    assert A.pick_cpus(0) == [8, 9, 10, 11]
    layout = A.cpu_layout([8, 9, 10, 11])
    assert layout["physical_cores"] == 4 and layout["smt_siblings"] == [32, 33, 34, 35] and not layout["whole_cores"]


def test_an_idle_job_leaves_a_domain_other_tenants_moved_onto(tmp_path, monkeypatch):
    allowed = make_tree(tmp_path)
    monkeypatch.setattr(A, "SYS_CPU", tmp_path)
    real_l3, real_numa = A.l3_domains, A.numa_of_cpu
    monkeypatch.setattr(A.os, "sched_getaffinity", lambda pid: allowed)
    monkeypatch.setattr(A, "l3_domains", lambda allowed=None, root=tmp_path: real_l3(allowed, root))
    monkeypatch.setattr(A, "numa_of_cpu", lambda cpu, root=tmp_path: real_numa(cpu, root))
    busy = {c: 0.0 for c in range(48)}
    monkeypatch.setattr(A, "_busy", lambda cpus, w: {c: busy.get(c, 0.0) for c in cpus})
    assert A.quieter_domain([4, 5, 6, 7], 0) is None                # nobody else there: stay
    busy.update({c + 24: 0.6 for c in (4, 5, 6, 7)})                 # a tenant on the siblings
    assert A.quieter_domain([4, 5, 6, 7], 0) == [8, 9, 10, 11]
    busy.update({c + 24: 0.0 for c in (4, 5, 6, 7)})
    busy[5] = 0.9                                                    # one CPU's worth on a core of ours
    assert A.quieter_domain([4, 5, 6, 7], 0) == [8, 9, 10, 11]
    busy[5] = 0.3                                                    # a little: not worth moving
    assert A.quieter_domain([4, 5, 6, 7], 0) is None
    busy.update({c + 24: 0.6 for c in (4, 5, 6, 7)})
    assert A.quieter_domain([4, 5, 6, 7], 0, exclude=[8]) is None    # the API server's domain: not that one
    busy.update({c: 0.5 for c in (8, 9, 10, 11)})                    # the alternative is no better
    assert A.quieter_domain([4, 5, 6, 7], 0) is None


def test_a_busy_job_moves_when_other_tenants_share_its_domain(tmp_path, monkeypatch):
    """Mid-run: the domain's busy time minus the job's own CPU time is other tenants' load.
    Two windows in a row at half a CPU or more and a domain carrying under half as much: move;
    the job's own load never counts; at most two moves."""
    import types

    allowed = make_tree(tmp_path)
    monkeypatch.setattr(A, "SYS_CPU", tmp_path)
    real_l3, real_numa = A.l3_domains, A.numa_of_cpu
    monkeypatch.setattr(A.os, "sched_getaffinity", lambda pid: allowed)
    monkeypatch.setattr(A, "l3_domains", lambda allowed=None, root=tmp_path: real_l3(allowed, root))
    monkeypatch.setattr(A, "numa_of_cpu", lambda cpu, root=tmp_path: real_numa(cpu, root))
    clock = {"t": 0.0, "own": 0}
    busy = {c: 0.0 for c in range(48)}
    monkeypatch.setattr(A, "time", types.SimpleNamespace(perf_counter=lambda: clock["t"]))
    monkeypatch.setattr(A, "cpu_snapshot", lambda: None)
    monkeypatch.setattr(A, "busy_between", lambda a, b, cpus: {c: busy.get(c, 0.0) for c in cpus})
    monkeypatch.setattr(A, "proc_cpu_ns", lambda pid: clock["own"])

    w = A.ContentionWatch([4, 5, 6, 7], [1], numa=0, exclude=[12])

    def window(own_cpus: float):     # 0.1 s in which the job itself used `own_cpus` CPUs
        clock["t"] += 0.1
        clock["own"] += int(own_cpus * 0.1e9)
        return w.check()

    assert w.check() == (0.0, None)
    busy.update({c: 0.9 for c in (4, 5, 6, 7)})                       # the job's own 3.6 CPUs
    f, to = window(3.6)
    assert abs(f) < 1e-6 and to is None
    busy.update({c + 24: 0.5 for c in (4, 5)})                         # a tenant on two siblings
    f, to = window(3.6)
    assert abs(f - 1.0) < 1e-6 and to is None                          # one window: not yet
    f, to = window(3.6)
    assert to == [8, 9, 10, 11]                                        # second: move (not CPU 0's, not the API server's)
    busy.update({c: 0.3 for c in (8, 9, 10, 11)})                      # the job is there now (own load only)
    w.cpus = to
    for _ in range(3):
        assert window(1.2)[1] is None
    busy.update({c: 0.6 for c in (8, 9, 10, 11)})                      # 1.2 CPUs of foreign load...
    busy.update({c: 0.4 for c in (16, 17, 18, 19, 20, 21, 22, 23)})    # ...and the rest of the socket
    busy.update({c: 0.4 for c in (4, 5, 6, 7)})                        # is no quieter: stay
    assert window(1.2)[1] is None and window(1.2)[1] is None
