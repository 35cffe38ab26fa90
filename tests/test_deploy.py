"""deploy/ manifests agree with the code they run: every argument is one the CLI accepts, the
policy ConfigMap loads, and the KubeSchedulerConfiguration's verbs and managed resources are
the routes and resource names the extender serves (reference deploy/*.yaml, README.md:43-58)."""
import json
from pathlib import Path

import yaml

from nanogpu import cli
from nanogpu.affinity import available_cores, busy_poll_fits
from nanogpu import types as T
from nanogpu.agent import node as agent
from nanogpu.config.policy import parse_policy
from nanogpu.extender.server import Router

DEPLOY = Path(__file__).resolve().parent.parent / "deploy"


def _docs(name):
    return [d for d in yaml.safe_load_all((DEPLOY / name).read_text()) if d]


def _container(name, kind):
    obj = next(d for d in _docs(name) if d["kind"] == kind)
    return obj["spec"]["template"]["spec"]["containers"][0]


def _mib(q: str) -> float:
    units = {"Ki": 1 / 1024, "Mi": 1, "Gi": 1024}
    for u, f in units.items():
        if q.endswith(u):
            return float(q[:-2]) * f
    return float(q) / 2 ** 20


def test_extender_memory_covers_the_shm_ledger_and_the_workers():
    """the /dev/shm emptyDir (Memory medium) is charged to the container's memory
    limit. The ledger at the deployment's geometry must fit the emptyDir's sizeLimit, and the
    limit must hold the sizeLimit plus the workers' own memory (~200 MiB each, plus the pod
    informer's reduced store: 200 MiB at 100k pods)."""
    from nanogpu import _native as N

    dep = next(d for d in _docs("nano-gpu-scheduler-amd.yaml") if d["kind"] == "Deployment")
    pod = dep["spec"]["template"]["spec"]
    c = pod["containers"][0]
    cfg = cli.parse(c["args"])
    ledger_mib = N.Ledger("", cfg.max_nodes, cfg.max_pods, True).bytes / 2 ** 20
    shm = next(v for v in pod["volumes"] if v["name"] == "shm")["emptyDir"]
    assert shm["medium"] == "Memory" and ledger_mib <= _mib(shm["sizeLimit"])
    limit = _mib(c["resources"]["limits"]["memory"])
    assert limit >= _mib(shm["sizeLimit"]) + cfg.workers * 200 + 200 + 512


def test_extender_deployment_args_parse():
    c = _container("nano-gpu-scheduler-amd.yaml", "Deployment")
    assert c["command"][-2:] == ["-m", "nanogpu"]
    cfg = cli.parse(c["args"])
    assert cfg.priority == "binpack" and cfg.workers == 2 and cfg.leader_elect
    assert cfg.frontend_threads == 1 and cfg.busy_poll_us == 8 and cfg.cpu_affinity == "auto"
    # the CPU request holds every busy-polling thread (else the server turns polling off)
    cpu = float(c["resources"]["requests"]["cpu"])
    # Guaranteed QoS, whole CPUs: what the static CPU manager needs to give the pod exclusive cores
    assert c["resources"]["limits"] == c["resources"]["requests"] and cpu == int(cpu)
    assert busy_poll_fits(cfg.workers, cfg.frontend_threads, cpu)
    ports = {p["containerPort"] for p in c.get("ports", [])}
    env = {e["name"]: e.get("value") for e in c.get("env", [])}
    assert int(env.get("PORT", 39999)) in ports or not ports


def test_agent_daemonset_args_parse():
    c = _container("nano-gpu-agent-amd.yaml", "DaemonSet")
    assert c["command"][:3] == ["python3", "-m", "nanogpu.agent"]
    a = agent.build_parser().parse_args(c["command"][3:] + (c.get("args") or []))
    assert a.selftest and a.calibrate and a.metrics_port == 9410


def test_policy_configmap_loads():
    cm = next(d for d in _docs("policy-configmap.yaml") if d["kind"] == "ConfigMap")
    spec = parse_policy(cm["data"]["policy.yaml"])
    assert {name for name, _ in spec.metrics} >= {"gpu_core_usage_avg", "gpu_memory_usage_avg",
                                                  T.GPU_HBM_ACTIVITY_METRIC}
    assert spec.metrics_scope == "cluster"
    for name, q in spec.metrics:      # every metric can be polled cluster-wide, by the exporter's labels
        assert q.cluster and "{node}" not in q.cluster and q.node_labels == ("hostname",)
        assert q.card_labels == ("gpu_id",)


def test_scheduler_config_matches_the_served_routes():
    ext = _docs("kube-scheduler-config.yaml")[0]["extenders"][0]
    assert ext["nodeCacheCapable"] is True
    prefix = "/" + ext["urlPrefix"].split("/", 3)[3]
    paths = {path for (method, path) in Router(None).table if method == "POST"}
    for verb in ("filterVerb", "prioritizeVerb", "bindVerb", "preemptVerb"):
        path = f"{prefix}/{ext[verb]}"
        assert path in paths, path
    assert {r["name"] for r in ext["managedResources"]} == {T.RESOURCE_GPU_PERCENT, T.RESOURCE_GPU_MEMORY}
    legacy = json.loads((DEPLOY / "scheduler-policy.json").read_text())["extenders"][0]
    assert legacy["filterVerb"] == ext["filterVerb"] and legacy["bindVerb"] == ext["bindVerb"]


def test_busy_poll_guard_reads_the_cgroup_quota(tmp_path, monkeypatch):
    from nanogpu import app

    (tmp_path / "cpu.max").write_text("400000 100000\n")          # limits.cpu: 4
    assert available_cores(tmp_path) <= 4.0
    monkeypatch.setattr("nanogpu.affinity.available_cores", lambda *a: 4.0)
    cfg = app.Config(workers=4, frontend_threads=2, busy_poll_us=20)
    app.guard_busy_poll(cfg)
    assert cfg.busy_poll_us == 0                                   # 12 cores needed
    monkeypatch.setattr("nanogpu.affinity.available_cores", lambda *a: 6.0)
    cfg = app.Config(workers=2, frontend_threads=2, busy_poll_us=20)
    app.guard_busy_poll(cfg)
    assert cfg.busy_poll_us == 20


def test_extender_flags_reach_the_config():
    """Round-3 switches: the label-less bind, the aiohttp pod watch, the writer mode; and their
    defaults (the reference's label contract, the native watch thread, the evented writer)."""
    base = cli.parse([])
    assert base.assume_label and base.native_pod_watch and base.bind_writer_mode == "evented"
    cfg = cli.parse(["--no-assume-label", "--no-native-pod-watch", "--bind-writer-mode", "threads"])
    assert not cfg.assume_label and not cfg.native_pod_watch and cfg.bind_writer_mode == "threads"
