"""Summarises a rocprofv3 SQLite output (`*_results.db`) into a markdown table for profiles/.

Usage: python tools/rocpd_summary.py gpurun_out/prof/probe_results.db [--title T] > profiles/x.md
"""
from __future__ import annotations

import argparse
import sqlite3


def summarise(db: str, title: str) -> str:
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    lines = [f"# {title}", "", f"Source: `rocprofv3 --kernel-trace --stats` → `{db}`", "",
             "| kernel | calls | total µs | avg µs | % GPU time |", "|---|---:|---:|---:|---:|"]
    for name, calls, tot, avg, pct in rows:
        lines.append(f"| `{name.replace('(anonymous namespace)::', '')[:110]}` | {calls} | {tot:.1f} | {avg:.2f} | {pct:.2f} |")
    shape = list(c.execute(
        "select name, grid_x, workgroup_x, vgpr_count, accum_vgpr_count, sgpr_count, lds_size, "
        "count(*), min(duration), max(duration) from kernels group by name, grid_x order by name"))
    lines += ["", "| kernel | grid_x (threads) | wg | vgpr | agpr | sgpr | lds B | n | min µs | max µs |",
              "|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|"]
    for r in shape:
        name = r[0].replace("(anonymous namespace)::", "").split("(")[0][:60]
        lines.append(f"| `{name}` | {r[1]} | {r[2]} | {r[3]} | {r[4]} | {r[5]} | {r[6]} | {r[7]} | "
                     f"{r[8] / 1e3:.1f} | {r[9] / 1e3:.1f} |")
    return "\n".join(lines) + "\n"


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--title", default="rocprofv3 kernel summary")
    a = ap.parse_args()
    print(summarise(a.db, a.title), end="")


if __name__ == "__main__":
    main()
