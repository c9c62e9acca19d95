#!/usr/bin/env python3
"""Per-kernel PMC summary from a rocprofv3 --pmc results database (rocpd sqlite).

    python scripts/pmc_summary.py gpurun_out/pmc/p1/run_results.db [name-filter ...]

Sums every counter over its instances for each dispatch, then averages over the
dispatches of each kernel (median dispatch duration alongside). Derived rows
(when the counters are present): effective clock = GRBM_GUI_ACTIVE / 8 XCDs /
duration, VALU issue share = SQ_ACTIVE_INST_VALU / SQ_BUSY_CYCLES-per-SIMD, VALU
instructions per wave, and the WAIT/ACTIVE split of SQ_WAVE_CYCLES
(MI355X_MICROARCH.md 'rocprofv3 PMC slots').
"""
import collections
import sqlite3
import statistics
import sys


def main():
    db = sys.argv[1]
    filters = sys.argv[2:]
    c = sqlite3.connect(db)
    rows = c.execute(
        "select dispatch_id, name, counter_name, counter_value, start, end from pmc_events"
    ).fetchall()
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    meta = {}
    for disp, name, cname, val, start, end in rows:
        per[disp][cname] += float(val)
        meta[disp] = (name, (end - start) * 1e-9)
    by_kernel = collections.defaultdict(list)
    for disp, counters in per.items():
        name, dur = meta[disp]
        if filters and not any(f in name for f in filters):
            continue
        by_kernel[name].append((dur, counters))
    for name, items in by_kernel.items():
        durs = [d for d, _ in items]
        keys = sorted({k for _, cs in items for k in cs})
        avg = {k: statistics.mean(cs.get(k, 0.0) for _, cs in items) for k in keys}
        dur = statistics.median(durs)
        print(f"== {name[:150]}")
        print(f"   dispatches {len(items)}, median duration {dur * 1e3:.3f} ms")
        for k in keys:
            print(f"   {k:24s} {avg[k]:.4g}")
        if "GRBM_GUI_ACTIVE" in avg and dur > 0:
            print(f"   effective clock          {avg['GRBM_GUI_ACTIVE'] / 8 / dur / 1e9:.3f} GHz")
        if "SQ_WAVE_CYCLES" in avg and avg["SQ_WAVE_CYCLES"] > 0:
            wc = avg["SQ_WAVE_CYCLES"]
            for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if k in avg:
                    print(f"   {k + ' / WAVE_CYCLES':40s} {avg[k] / wc:.3f}")
        if "SQ_INSTS_VALU" in avg and avg.get("SQ_WAVES"):
            print(f"   VALU instructions per wave {avg['SQ_INSTS_VALU'] / avg['SQ_WAVES']:.4g}")


if __name__ == "__main__":
    main()
