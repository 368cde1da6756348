#!/usr/bin/env python3
"""Per-kernel and per-copy-kind totals from a rocprofv3 SQLite (rocpd) database -> Markdown.

    python tools/rocpd_summary.py gpurun_out/dlprof/dl_results.db > profiles/x.md
"""
import sqlite3
import sys


def main(path: str) -> None:
    db = sqlite3.connect(path)
    print(f"# rocprofv3 summary of `{path.split('/')[-1]}`\n")
    print("## Kernels\n\n| kernel | calls | total ms | avg us | % |\n|---|---:|---:|---:|---:|")
    rows = list(db.execute("select name, count(*), sum(duration) from kernels group by name order by 3 desc"))
    tot = sum(r[2] for r in rows) or 1
    for name, n, d in rows:
        short = name.split("(")[0][:90]
        print(f"| `{short}` | {n} | {d / 1e6:.3f} | {d / n / 1e3:.2f} | {100 * d / tot:.1f} |")
    print("\n## Memory copies\n\n| kind | calls | total MB | total ms | GB/s |\n|---|---:|---:|---:|---:|")
    for name, n, sz, d in db.execute(
            "select name, count(*), sum(size), sum(duration) from memory_copies group by name order by 4 desc"):
        print(f"| {name} | {n} | {sz / 1e6:.1f} | {d / 1e6:.3f} | {sz / max(d, 1):.2f} |")


if __name__ == "__main__":
    main(sys.argv[1])
