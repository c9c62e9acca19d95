"""Summarise a rocprofv3 CSV output directory (scripts/profile.sh) as markdown:
top kernels by total time and, when a marker trace is present, the host-side
roctx ranges of the mxs runtime (halo.*, stencil.*, pingpong.*)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def _rows(pattern):
    files = sorted(glob.glob(pattern, recursive=True))
    if not files:
        return []
    with open(files[0], newline="") as f:
        return list(csv.DictReader(f))


def _db_stats(d):
    """Per-kernel stats from a rocpd SQLite database (rocprofv3's default output
    on newer images), in the shape of kernel_stats.csv rows, plus each kernel's
    VGPR / LDS / scratch resources."""
    import sqlite3

    dbs = sorted(glob.glob(os.path.join(d, "**", "*.db"), recursive=True))
    if not dbs:
        return []
    c = sqlite3.connect(dbs[0])
    q = ("select name, count(*), sum(duration), avg(duration), min(duration), max(duration), max(vgpr_count), "
         "max(accum_vgpr_count), max(lds_size), max(scratch_size) from kernels group by name")
    return [{"Name": n, "Calls": k, "TotalDurationNs": t, "AverageNs": a, "MinNs": lo, "MaxNs": hi, "VGPR": v,
             "AGPR": ag, "LDS": lds, "Scratch": sc} for n, k, t, a, lo, hi, v, ag, lds, sc in c.execute(q)]


def main(d: str) -> int:
    ks = _rows(os.path.join(d, "**", "*kernel_stats.csv"))
    from_db = False
    if not ks:
        ks = _db_stats(d)
        from_db = bool(ks)
    print(f"# Profile summary: {os.path.basename(os.path.normpath(d))}\n")
    if from_db:
        total = sum(float(r["TotalDurationNs"]) for r in ks)
        print("(rocpd database; min / max per kernel and its resources as dispatched)\n")
        print("| kernel | calls | total ms | avg us | min us | max us | % | VGPR | LDS B | scratch B |")
        print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
        for r in sorted(ks, key=lambda r: -float(r["TotalDurationNs"]))[:15]:
            name = r["Name"]
            name = name if len(name) < 110 else name[:107] + "..."
            print(f"| `{name}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.3f} | "
                  f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['MinNs']) / 1e3:.1f} | {float(r['MaxNs']) / 1e3:.1f} | "
                  f"{100 * float(r['TotalDurationNs']) / total:.1f} | {r['VGPR']} | {r['LDS']} | {r['Scratch']} |")
        return 0
    if ks:
        total = sum(float(r["TotalDurationNs"]) for r in ks)
        print("| kernel | calls | total ms | avg us | % |")
        print("|---|---:|---:|---:|---:|")
        for r in sorted(ks, key=lambda r: -float(r["TotalDurationNs"]))[:15]:
            name = r["Name"]
            name = name if len(name) < 110 else name[:107] + "..."
            print(f"| `{name}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.3f} | "
                  f"{float(r['AverageNs']) / 1e3:.1f} | {100 * float(r['TotalDurationNs']) / total:.1f} |")
    mk = _rows(os.path.join(d, "**", "*marker_api_stats.csv"))
    if mk:
        print("\n| roctx range | count | total ms (host) | avg us |")
        print("|---|---:|---:|---:|")
        for r in sorted(mk, key=lambda r: -float(r["TotalDurationNs"])):
            print(f"| {r['Name']} | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.3f} | "
                  f"{float(r['AverageNs']) / 1e3:.1f} |")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
