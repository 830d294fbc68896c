#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd SQLite database (kernel trace) into a Markdown table.

usage: rocpd_summary.py <results.db> [title] > profiles/<name>.md
"""
import re
import sqlite3
import sys


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name)
    return name if len(name) < 90 else name[:87] + "..."


def main():
    db = sqlite3.connect(sys.argv[1])
    title = sys.argv[2] if len(sys.argv) > 2 else sys.argv[1]
    rows = db.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration), "
                      "max(grid_x), max(workgroup_x), max(vgpr_count), max(accum_vgpr_count), max(lds_size), "
                      "max(scratch_size) from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    print(f"# {title}\n")
    print("rocprofv3 --kernel-trace --stats (durations in microseconds)\n")
    print("| kernel | calls | total us | avg us | min us | max us | % | grid | wg | vgpr | agpr | lds B | scratch B |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|---|")
    for r in rows:
        print(f"| `{short(r[0])}` | {r[1]} | {r[2] / 1e3:.1f} | {r[3] / 1e3:.2f} | {r[4] / 1e3:.2f} | {r[5] / 1e3:.2f} | "
              f"{100.0 * r[2] / total:.1f} | {r[6]} | {r[7]} | {r[8]} | {r[9]} | {r[10]} | {r[11]} |")


if __name__ == "__main__":
    main()
