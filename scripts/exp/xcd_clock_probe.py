"""Are the per-XCD shader clocks of the headline pass stable from pass to pass? (round 6)

A balanced pass ends with its slowest XCD (profiles/r06_fill). If each XCD's
clock relative to the others held from one pass to the next, shares sized in
proportion to the previous pass's per-XCD clocks would end every XCD together.
This stamps `--passes` back-to-back 32768^2 passes (S = 20, sum form, after
~200 ms of warm passes) and prints, per pass, each XCD's median clock, and the
pass time a clock-proportional split would have given (the total work over the
summed per-XCD rates) against the balanced split's (the slowest XCD): with the
CURRENT pass's clocks (the ceiling) and with the PREVIOUS pass's (what a
feedback scheme could get).

usage: python scripts/exp/xcd_clock_probe.py [--passes 24] [--size 32768]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from cuda_mpi_scratch_amd import core, hip  # noqa: E402
from cuda_mpi_scratch_amd.utils.cycles import stamped_passes  # noqa: E402


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--passes", type=int, default=24)
    p.add_argument("--size", type=int, default=32768)
    args = p.parse_args()
    n, S = args.size, 20
    g = core().TileGeom.aligned(n, n, S, S, 4)
    a = torch.rand(g.alloc_elems(), device="cuda", dtype=torch.float32)
    b = torch.empty_like(a)
    s = torch.cuda.current_stream().cuda_stream

    def launch():
        hip().stencil5_tb(a.data_ptr(), b.data_ptr(), g, S, 0, n, 0, n, 0.2, 0.2, True, "f32", s, "auto", True)

    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.2:
        launch()
        torch.cuda.synchronize()
    rows = stamped_passes(launch, s, args.passes, warm=2)
    prev = None
    gain_now, gain_prev = [], []
    for i, r in enumerate(rows):
        mhz = r["xcd_mhz"]
        rates = list(mhz.values())
        slow = min(rates)
        now = slow * len(rates) / sum(rates)  # proportional split / balanced split, same clocks
        rec = {"pass": i, "us": round(r["us"], 1), "xcd_mhz": {k: round(v) for k, v in mhz.items()},
               "proportional_now": round(now, 4)}
        if prev is not None and set(prev) == set(mhz):
            # shares from the previous pass's clocks p, run at this pass's r: XCD k
            # ends at (p_k / sum p) / r_k of the work; relative to the balanced split
            # (1/n) / r_min
            sp = sum(prev.values())
            t = max((prev[k] / sp) / mhz[k] for k in mhz) * len(rates) * slow
            rec["proportional_prev"] = round(t, 4)
            gain_prev.append(t)
        gain_now.append(now)
        prev = mhz
        print(json.dumps(rec), flush=True)
    # One calibration for the box: shares from the mean clocks over all passes.
    keys = sorted(rows[0]["xcd_mhz"])
    mean = {k: statistics.mean(r["xcd_mhz"][k] for r in rows if k in r["xcd_mhz"]) for k in keys}
    sm = sum(mean.values())
    fixed = []
    for r in rows:
        mhz = r["xcd_mhz"]
        if set(mhz) != set(mean):
            continue
        fixed.append(max((mean[k] / sm) / mhz[k] for k in mhz) * len(mhz) * min(mhz.values()))
    print(json.dumps({"summary": True, "proportional_now_median": round(statistics.median(gain_now), 4),
                      "proportional_prev_median": round(statistics.median(gain_prev), 4) if gain_prev else None,
                      "proportional_fixed_median": round(statistics.median(fixed), 4) if fixed else None,
                      "mean_xcd_mhz": {k: round(v) for k, v in mean.items()}}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
