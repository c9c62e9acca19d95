"""Summary of scripts/exp/opening_probe.py outputs: per solver the choice, and per
candidate outer set the median of its per-round ratios by GPU events (what the
decision uses) and by the host clock (enqueue to drained, as the window is
timed), with the number of rounds above 1.2 (a serialised opening).

usage: python scripts/exp/opening_summary.py FILE [FILE ...]"""
import json
import statistics
import sys


def main() -> int:
    for path in sys.argv[1:]:
        print(f"== {path}")
        for line in open(path):
            if not line.startswith("{"):
                continue
            d = json.loads(line)
            if "solver" not in d:
                print("  ", {k: v for k, v in d.items() if k != "median_phases"})
                continue
            print(f"  solver {d['solver']}: {d['opening']}, ratio {d['ratio']:.3f}, lead {d.get('lead_us', 0):.1f} us")
            host = dict((w, r) for w, r in d.get("local_host_candidate_ratios", []))
            for w, r in d.get("local_candidate_ratios", []):
                h = host.get(w, [])
                print(f"     outer {w:3d}: events median {statistics.median(r):.3f} (>1.2: {sum(x > 1.2 for x in r):2d})"
                      + (f"   host median {statistics.median(h):.3f} (>1.2: {sum(x > 1.2 for x in h):2d})" if h else ""))
    return 0


if __name__ == "__main__":
    sys.exit(main())
