#!/usr/bin/env python3
"""Device frees inside the solver's prepare() / warm().

    python scripts/hip_free_check.py DIR

DIR holds a rocprofv3 run with ``--hip-trace --marker-trace --output-format csv``
(``*hip_api_trace.csv`` and ``*marker_api_trace.csv``). Prints every roctx range
named ``stencil.prepare`` / ``stencil.warm`` / ``stencil.run`` and every
``hipFree*`` call, and counts the frees that fall between the first
``stencil.prepare`` start and the last ``stencil.warm`` end (the stretch between
construction and a bench window). A free there starts the driver's wipe of the
freed VRAM, which slows HBM reads for a while (profiles/r05_free_state).
"""
import csv
import glob
import os
import sys


def rows(pattern):
    out = []
    for path in glob.glob(pattern, recursive=True):
        with open(path, newline="") as f:
            out += list(csv.DictReader(f))
    return out


def col(r, *names):
    for n in names:
        for k in r:
            if k.lower() == n.lower():
                return r[k]
    return None


def main() -> int:
    d = sys.argv[1] if len(sys.argv) > 1 else "."
    hip = rows(os.path.join(d, "**", "*hip_api_trace.csv"))
    marks = rows(os.path.join(d, "**", "*marker_api_trace.csv"))
    if not hip:
        print(f"no hip_api_trace.csv under {d}")
        return 2
    frees = [(int(col(r, "Start_Timestamp")), col(r, "Function")) for r in hip
             if (col(r, "Function") or "").startswith("hipFree")]
    ranges = []
    for r in marks:
        name = col(r, "Function", "Message", "Name") or ""
        if name.startswith("stencil.") and name.split(".")[1] in ("prepare", "warm", "run"):
            ranges.append((int(col(r, "Start_Timestamp")), int(col(r, "End_Timestamp")), name))
    ranges.sort()
    prep = [r for r in ranges if r[2] == "stencil.prepare"]
    warm = [r for r in ranges if r[2] == "stencil.warm"]
    print(f"hip API calls {len(hip)}, hipFree* {len(frees)}, ranges: prepare {len(prep)}, warm {len(warm)}, "
          f"run {sum(1 for r in ranges if r[2] == 'stencil.run')}")
    if not prep or not warm:
        print("no stencil.prepare / stencil.warm ranges (marker trace missing?)")
        return 2
    t0, t1 = prep[0][0], warm[-1][1]
    inside = [f for f in frees if t0 <= f[0] <= t1]
    for t, fn in frees:
        where = "INSIDE prepare..warm" if t0 <= t <= t1 else ("before" if t < t0 else "after")
        print(f"  {fn} at {(t - t0) / 1e6:+.3f} ms from the first prepare: {where}")
    print(f"frees between the first prepare() and the last warm(): {len(inside)}")
    return 1 if inside else 0


if __name__ == "__main__":
    sys.exit(main())
