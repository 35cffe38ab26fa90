"""Markdown rows for bench --json-out files: value, p50 bind, extender CPU (+ by thread), the
rank's and API server's CPUs and how busy they and their SMT siblings were while timed.
usage: python tools/summarize_runs.py FILE.json [...]"""
import json
import statistics
import sys


def main(paths: list[str]) -> None:
    vals = []
    print("| run | pods/s | p50 bind ms | CPU us/pod (fe / wr / watch / loop) | rank CPUs | busy % rank / siblings / apiserver / siblings / host |")
    print("|---|---:|---:|---|---|---|")
    for p in paths:
        d = json.load(open(p))
        g = d.get("diagnostics", {})
        th = g.get("extender_cpu_us_per_pod_by_thread_rank0") or {}
        b = d.get("cpu_busy_pct_rank0") or {}
        vals.append(d["value"])
        cpus = d["config"].get("cpus_rank0", "")
        cpus = cpus.split(",")[0] + "-" + cpus.split(",")[-1] if "," in cpus else cpus
        print(f"| {p.rsplit('/', 1)[-1]} | {d['value']:,.0f} | {d['p50_bind_ms']} | {d['extender_cpu_us_per_pod_rank0']} "
              f"({th.get('ngpu-fe')} / {th.get('ngpu-wr-io', '-')} / {th.get('ngpu-podwatch')} / {th.get('main')}) | "
              f"{cpus} | {b.get('rank')} / {b.get('rank_smt_siblings')} / {b.get('apiserver')} / "
              f"{b.get('apiserver_smt_siblings')} / {b.get('host')} |")
    if len(vals) > 1:
        m = statistics.median(vals)
        print(f"\nmedian {m:,.0f} pods/s; each run vs the median: "
              + ", ".join(f"{100 * (v / m - 1):+.1f} %" for v in vals))


if __name__ == "__main__":
    main(sys.argv[1:])
