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


def main(d: str) -> int:
    ks = _rows(os.path.join(d, "**", "*kernel_stats.csv"))
    print(f"# Profile summary: {os.path.basename(os.path.normpath(d))}\n")
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
