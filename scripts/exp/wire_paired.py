"""Rehearsed wire time, measured as PAIRED in-process rounds.

Round 5's wire-delay tables ranked schedules on medians of 5 single-shot
processes each; their differences were smaller than the shot-to-shot spread
(the chip's clock, docs/PERF.md). Here every schedule runs in ONE process, and
every round times one window of each back to back (order rotated per round), so
the clock drift that moves single shots cancels in the per-round ratios.

The schedules are ONE loopback solver switched at run time
(StencilSolver::force_opening / force_steady), plus one fused solver built after
the loopback solver's prepare() (its decision and measured exchange lead are
taken with no other solver in the process): a process
holding four solvers (eight streams over GPU_MAX_HW_QUEUES = 4) ran the
interior-first schedules of some of them 1.5-1.8x slower than alone, while one
loopback solver beside the fused one ran them at their single-process speed
(profiles/r06_wire/README.md).

For each rehearsed wire time W (--wire-delay-us: a one-wave kernel holding the
stream W us after each RCCL transfer, the one-GPU stand-in for xGMI time), on a
rank tile through RCCL loopback in the peers' schedule:
  serial : exchange, then the pass;
  ifirst : interior-first (the outer set prepare() measured or modelled);
  fused  : the 1x1 periodic tile (the same window with no exchange at all);
  auto   : what prepare() decided (opening auto, the bench's default) -- one of
           the two; its ratios are that schedule's.
A round: ~100 ms of warm passes (the bench's clock warm-up), then for each
schedule one drained warm pass and one timed window (host clock, enqueue to
streams drained + torch.cuda.synchronize(), as bench.py times it).

Per W it prints the median paired ratios with IQR, the notch 1.58 IQR / sqrt(n)
and the interval median +- notch. An exchange is "hidden" only where the
interval of the decided schedule / fused contains 1.

--steady: 240-step windows (12 super-steps), the opening interior-first, the
later super-steps serial or interior-first (force_steady), against the fused
tile; "auto" is prepare()'s steady decision.

usage: python scripts/exp/wire_paired.py [--tile WxH] [--wires 0,20,40,80] [--rounds 16] [--steady]
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
from cuda_mpi_scratch_amd.parallel import init as dist_init  # noqa: E402


def stats(xs):
    xs = sorted(xs)
    n = len(xs)
    med = statistics.median(xs)
    q1, q3 = xs[n // 4], xs[(3 * n) // 4]
    notch = 1.58 * (q3 - q1) / math.sqrt(n)
    return {"median": round(med, 4), "iqr": round(q3 - q1, 4), "notch": round(notch, 4),
            "lo": round(med - notch, 4), "hi": round(med + notch, 4), "n": n}


def window(st, steps):
    """One bench-shaped window: drained streams, then host clock from the
    enqueue to the solver's streams drained + the device sync."""
    st.solver.warm(steps, 1)  # one untimed, state-preserving pass (the bench's warm tail)
    st.synchronize()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    st.run(steps)
    st.synchronize()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--tile", default="16384x8192")
    p.add_argument("--wires", default="0,20,40,80")
    p.add_argument("--rounds", type=int, default=16)
    p.add_argument("--steady", action="store_true")
    p.add_argument("--warm-ms", type=float, default=100.0)
    args = p.parse_args()
    ctx = dist_init(backend="nccl")
    hip().set_comm_timeout(120.0)
    w, h = (int(v) for v in args.tile.split("x"))
    steps = 240 if args.steady else 20
    base = dict(global_width=w, global_height=h, dims="1x1", dtype="f32", time_block=20)
    for wire in [float(x) for x in args.wires.split(",")]:
        kw = dict(opening="interior-first", steady="auto") if args.steady else dict(opening="auto")
        st = Stencil2D(StencilConfig(**base, backend="rccl", loopback=True, rehearse_peers=True, wire_delay_us=wire,
                                     **kw), ctx)
        st.run(steps)
        st.prepare(steps)  # the decision (opening, or steady with --steady), before any other solver exists
        # The fused solver is built after the decision: with it alive during prepare() the measured
        # exchange lead came out 2x too long at 20 and 80 us of wire (profiles/r06_wire/README.md).
        fused = Stencil2D(StencilConfig(**base), ctx)
        fused.run(steps)
        fused.prepare(steps)
        choice = st.solver.schedule_times()
        decided = choice["steady"] if args.steady else choice["opening"]
        force = st.solver.force_steady if args.steady else st.solver.force_opening
        names = ["serial", "ifirst", "fused"]
        ms = {k: [] for k in names}
        for r in range(args.rounds):
            fused.warm(steps, args.warm_ms / 1e3)  # the bench's clock warm-up, once per round
            order = names[r % len(names):] + names[:r % len(names)]
            for k in order:
                if k == "fused":
                    ms[k].append(window(fused, steps))
                else:
                    force("serial" if k == "serial" else "interior-first")
                    ms[k].append(window(st, steps))
        force("auto")
        auto = "ifirst" if decided == "interior-first" else "serial"

        def ratio(a, b):
            return stats([x / y for x, y in zip(ms[a], ms[b])])

        rec = {"tile": args.tile, "steps": steps, "wire_us": wire, "rounds": args.rounds,
               "schedule": "steady" if args.steady else "opening", "decided": decided, "auto_is": auto,
               "decision": {"reason": choice["steady_reason"] if args.steady else choice["reason"],
                            "opening_ratio": round(choice["ratio"], 3), "outer_wgs": choice["outer_wgs"],
                            "lead_us": round(choice["lead_us"], 1)},
               "side_stream": st.solver.stream_note(),
               "median_ms": {k: round(statistics.median(v), 4) for k, v in ms.items()},
               "ratios": {"ifirst/serial": ratio("ifirst", "serial"), "serial/fused": ratio("serial", "fused"),
                          "ifirst/fused": ratio("ifirst", "fused"), "auto/fused": ratio(auto, "fused")},
               "ms": {k: [round(x, 4) for x in v] for k, v in ms.items()}}
        print(json.dumps(rec), flush=True)
        st.synchronize()
        fused.synchronize()
        del st, fused
        torch.cuda.synchronize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
