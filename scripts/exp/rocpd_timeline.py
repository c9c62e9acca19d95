"""Per-window kernel timeline (markdown) from a rocprofv3 SQLite database: the
trace is cut into windows at idle gaps longer than --gap-us; the last --windows
windows are listed kernel by kernel (start / end relative to the window's first
kernel), plus the median span of every window.

usage: python scripts/exp/rocpd_timeline.py <results.db> [--gap-us 1000] [--windows 2]"""
import argparse
import sqlite3


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("db")
    p.add_argument("--gap-us", type=float, default=1000.0)
    p.add_argument("--windows", type=int, default=2)
    a = p.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name}, start, end from kernels order by start").fetchall()
    wins, cur = [], []
    for r in rows:
        if cur and r[1] - max(x[2] for x in cur) > a.gap_us * 1e3:
            wins.append(cur)
            cur = []
        cur.append(r)
    if cur:
        wins.append(cur)
    spans = sorted((max(x[2] for x in w) - w[0][1]) / 1e3 for w in wins[1:])
    print(f"# kernel timeline: {a.db}\n")
    print(f"{len(wins)} windows (split at idle gaps > {a.gap_us:.0f} us); median span of windows 2..: "
          f"{spans[len(spans) // 2]:.1f} us\n" if spans else "")
    for k, w in enumerate(wins[-a.windows:]):
        t0 = w[0][1]
        print(f"## window {len(wins) - a.windows + k} ({(max(x[2] for x in w) - t0) / 1e3:.1f} us)\n")
        print("| kernel | start us | end us | us |")
        print("|---|---|---|---|")
        for n, s, e in w:
            short = n if len(n) < 90 else n[:87] + "..."
            print(f"| `{short}` | {(s - t0) / 1e3:.1f} | {(e - t0) / 1e3:.1f} | {(e - s) / 1e3:.1f} |")
        print()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
