"""Level order A/B in the bench's own window (round 6: ascending at every share
length vs the round-5 rule, descending on shares past 768 rows).

One process, one solver per tile; each round sets the order
(hip().set_pipe_lag1: on = ascending everywhere, off = descending everywhere),
runs ~200 ms of warm passes and a drained warm pass, then times one window as
bench.py does (host clock, enqueue to drained + device sync) with clock stamps
around it: wall ms, the pass's shader cycles at the slowest XCD's clock and
the median clock. The order alternates first/second from round to round.
Prints per tile the paired ratios asc / desc (median, notch) of wall time and
of cycles.

usage: python scripts/exp/order_ab.py [--tiles 32768x32768,16384x16384] [--rounds 12] [--steps 20]
"""
import argparse
import json
import math
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from cuda_mpi_scratch_amd import hip  # noqa: E402
from cuda_mpi_scratch_amd.models.stencil2d import Stencil2D, StencilConfig  # noqa: E402


def notch(xs):
    xs = sorted(xs)
    n = len(xs)
    med = statistics.median(xs)
    iqr = xs[(3 * n) // 4] - xs[n // 4]
    nt = 1.58 * iqr / math.sqrt(n)
    return {"median": round(med, 4), "notch": round(nt, 4), "lo": round(med - nt, 4), "hi": round(med + nt, 4)}


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--tiles", default="32768x32768,16384x16384")
    p.add_argument("--rounds", type=int, default=12)
    p.add_argument("--steps", type=int, default=20)
    args = p.parse_args()
    H = hip()
    K = H.clock_stamp_slots()
    khz = H.wall_clock_rate_khz()
    stamps = torch.zeros(6 * K, dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    for tile in args.tiles.split(","):
        w, h = (int(v) for v in tile.split("x"))
        st = Stencil2D(StencilConfig(global_width=w, global_height=h, dims="1x1", dtype="f32"))
        st.run(args.steps)
        st.prepare(args.steps)
        res = {True: [], False: []}
        for r in range(args.rounds):
            for lag in ((True, False) if r % 2 == 0 else (False, True)):
                H.set_pipe_lag1(lag)
                st.warm(args.steps, 0.2, 1)
                st.synchronize()
                torch.cuda.synchronize()
                H.clock_stamp(stamps.data_ptr(), s)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                st.run(args.steps)
                st.synchronize()
                torch.cuda.synchronize()
                wall = (time.perf_counter() - t0) * 1e3
                used = bool(H.last_pipe_lag1())
                H.clock_stamp(stamps.data_ptr() + 3 * K * 8, s)
                torch.cuda.synchronize()
                v = stamps.cpu().view(2, K, 3).tolist()
                d0 = {int(x): (c, t) for x, c, t in v[0]}
                d1 = {int(x): (c, t) for x, c, t in v[1]}
                per = {}
                for x in set(d0) & set(d1):
                    if d1[x][1] > d0[x][1]:
                        per.setdefault(x >> 16, []).append((d1[x][0] - d0[x][0]) / ((d1[x][1] - d0[x][1]) / (khz / 1e3)))
                slow = min(statistics.median(m) for m in per.values())
                med = statistics.median([m for ms in per.values() for m in ms])
                res[lag].append({"wall_ms": wall, "kcycles_slowest": wall * 1e3 * slow / 1e3, "mhz": med,
                                 "mhz_slowest": slow, "lag1_used": used})
        H.set_pipe_lag1(True)
        a, d = res[True], res[False]
        rec = {"tile": tile, "steps": args.steps, "rounds": args.rounds,
               "asc_wall_ms": round(statistics.median(x["wall_ms"] for x in a), 4),
               "desc_wall_ms": round(statistics.median(x["wall_ms"] for x in d), 4),
               "asc_mhz": round(statistics.median(x["mhz"] for x in a)),
               "desc_mhz": round(statistics.median(x["mhz"] for x in d)),
               "wall_asc_over_desc": notch([x["wall_ms"] / y["wall_ms"] for x, y in zip(a, d)]),
               "kcycles_asc_over_desc": notch([x["kcycles_slowest"] / y["kcycles_slowest"] for x, y in zip(a, d)]),
               "mhz_asc_over_desc": notch([x["mhz"] / y["mhz"] for x, y in zip(a, d)]),
               "orders_used": [all(x["lag1_used"] for x in a), not any(x["lag1_used"] for x in d)],
               "kernel": H.last_stencil_dispatch()}
        print(json.dumps(rec), flush=True)
        del st
        torch.cuda.synchronize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
