"""Kernel summary (markdown) from a rocprofv3 SQLite (rocpd) database.

usage: python scripts/exp/rocpd_summary.py <results.db> [top_n]"""
import sqlite3
import sys


def main() -> int:
    db = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name}, count(*), sum(end - start), min(end - start), max(end - start) "
                     f"from kernels group by {name} order by sum(end - start) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    print(f"# kernel summary: {db}\n")
    print("| kernel | calls | total ms | % | median-free avg us | min us | max us |")
    print("|---|---|---|---|---|---|---|")
    for n, k, s, lo, hi in rows[:top]:
        short = n if len(n) < 110 else n[:107] + "..."
        print(f"| `{short}` | {k} | {s / 1e6:.3f} | {100 * s / total:.1f} | {s / k / 1e3:.1f} | {lo / 1e3:.1f} | {hi / 1e3:.1f} |")
    print(f"\n{len(rows)} distinct kernels, {sum(r[1] for r in rows)} dispatches, {total / 1e6:.2f} ms of kernel time")
    return 0


if __name__ == "__main__":
    sys.exit(main())
