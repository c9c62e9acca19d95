"""Summarise stencil_tune JSON lines: python scripts/tune_summary.py gpurun_out/tuneNN_*.log"""
import json
import sys

for path in sys.argv[1:]:
    print("==", path)
    for line in open(path):
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        if "mismatches" in d:
            if d["mismatches"]:
                print("MISMATCH", d)
            continue
        if "gcells_s" not in d:
            print(d)
            continue
        print(f"{d['variant']:32s} {d['gcells_s']:8.1f} {d['median_ms']:.3f}")
