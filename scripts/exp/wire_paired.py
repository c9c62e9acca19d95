"""Rehearsed wire time, measured as PAIRED in-process rounds.

Round 5's wire-delay tables ranked schedules on medians of 5 single-shot
processes each; their differences were smaller than the shot-to-shot spread
(the chip's clock, docs/PERF.md). Here every schedule runs in ONE process, on
the same tile, and every round times one window of each schedule back to back
(order rotated per round), so the clock drift that moves single shots cancels
in the per-round ratios.

For each rehearsed wire time W (--wire-delay-us: a one-wave kernel holding the
stream W us after each RCCL transfer, the one-GPU stand-in for xGMI time), on
the 8-GPU rank tile through RCCL loopback in the peers' schedule:
  serial  : opening = serial (exchange, then the pass);
  auto    : opening = auto (prepare() decides; the bench's default);
  ifirst  : (--forced) opening = interior-first, forced (outer set from the
            model). In a process holding several solvers it ran 1.5-1.8x slower
            than the same solver alone (0.29 ms in single-process windows,
            profiles/r06_wire), so its in-process ratios are not evidence;
and once, without any exchange:
  fused   : the 1x1 periodic tile (the window with no exchange at all).
A round: ~100 ms of warm passes (the bench's clock warm-up), then for each
schedule one drained warm pass and one timed window (host clock, enqueue to
streams drained + torch.cuda.synchronize(), as bench.py times it).

Per W it prints the median paired ratios (auto / serial, ifirst / serial,
auto / fused, serial / fused) with IQR and the notch 1.58 IQR / sqrt(n), and the
interval median +- notch: "hidden" is claimed only where the interval of
auto / fused contains 1 (the exchange costs nothing measurable) -- or lies
below the serial interval.

--steady: 240-step windows (12 super-steps) with the opening forced
interior-first and steady = serial / interior-first / auto (the later
super-steps), against the fused tile.

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
    p.add_argument("--forced", action="store_true", help="also the forced interior-first opening")
    args = p.parse_args()
    ctx = dist_init(backend="nccl")
    hip().set_comm_timeout(120.0)
    w, h = (int(v) for v in args.tile.split("x"))
    steps = 240 if args.steady else 20
    base = dict(global_width=w, global_height=h, dims="1x1", dtype="f32", time_block=20)
    if args.steady:
        modes = {"st_serial": dict(opening="interior-first", steady="serial"),
                 "st_ifirst": dict(opening="interior-first", steady="interior-first"),
                 "st_auto": dict(opening="interior-first", steady="auto")}
        ref = "st_serial"
    else:
        modes = {"serial": dict(opening="serial"), "auto": dict(opening="auto")}
        if args.forced:  # in a process with several solvers the forced opening ran 1.6x slower than alone (r06)
            modes["ifirst"] = dict(opening="interior-first")
        ref = "serial"
    fused = Stencil2D(StencilConfig(**base), ctx)
    fused.run(steps)
    fused.prepare(steps)
    for wire in [float(x) for x in args.wires.split(",")]:
        sts = {}
        for name, kw in modes.items():
            st = Stencil2D(StencilConfig(**base, backend="rccl", loopback=True, rehearse_peers=True,
                                         wire_delay_us=wire, **kw), ctx)
            st.run(steps)
            st.prepare(steps)
            sts[name] = st
        sts["fused"] = fused
        names = list(sts)
        ms = {k: [] for k in names}
        for r in range(args.rounds):
            fused.warm(steps, args.warm_ms / 1e3)  # the bench's clock warm-up, once per round
            order = names[r % len(names):] + names[:r % len(names)]
            for k in order:
                ms[k].append(window(sts[k], steps))
        rec = {"tile": args.tile, "steps": steps, "wire_us": wire, "rounds": args.rounds,
               "median_ms": {k: round(statistics.median(v), 4) for k, v in ms.items()}}
        ratios = {}
        for k in names:
            if k != ref:
                ratios[f"{k}/{ref}"] = stats([a / b for a, b in zip(ms[k], ms[ref])])
            if k != "fused":
                ratios[f"{k}/fused"] = stats([a / b for a, b in zip(ms[k], ms["fused"])])
        rec["ratios"] = ratios
        for k in names:
            if k == "fused":
                continue
            c = sts[k].solver.schedule_times()
            rec.setdefault("decision", {})[k] = {"opening": c["opening"], "steady": c["steady"],
                                                 "ratio": round(c["ratio"], 3), "outer_wgs": c["outer_wgs"],
                                                 "lead_us": round(c["lead_us"], 1),
                                                 "side_stream": sts[k].solver.stream_note()}
        rec["ms"] = {k: [round(x, 4) for x in v] for k, v in ms.items()}
        print(json.dumps(rec), flush=True)
        for st in list(sts.values()):
            if st is not fused:
                st.synchronize()
        del sts
        torch.cuda.synchronize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
