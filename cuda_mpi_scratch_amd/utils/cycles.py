"""Clock-independent cost of a kernel launch: shader cycles per pass.

The stencil passes are VALU-bound and the chip's shader clock follows its power
management (1.5-2.1 GHz under this load, docs/PERF.md "The clock, measured"),
so a pass's wall time moves by +-10% from box to box and run to run while its
cost in shader cycles stays within ~1%. Cycles are measured from two
``hip().clock_stamp`` launches around each pass (512 one-wave workgroups; each
records its XCD and CU, the CU's shader-clock counter ``s_memtime`` and the
global 100 MHz wall clock): the pass's wall span is the last "after" stamp minus
the first "before" stamp, and each CU seen in both stamps gives its own mean
clock over the span (counter delta / wall delta).

The 8 XCDs do not run at one clock: within one pass their median clocks
differ by 2-8% (profiles/r06_fill), and a balanced pass (equal cycles per
workgroup) ends when the slowest XCD's workgroups end. So the pass's cost is
span x the SLOWEST XCD's clock (``cycles``: the cycles the critical workgroups
ran, plus launch and drain); span x the median CU clock (``cycles_median_clock``)
also carries the XCD clock spread, which varies from run to run.

The regression tests (tests/test_gpu_cycles.py) hold these counts to budgets,
so a slower kernel body fails on any box, whatever clock it happens to run at.
"""
from __future__ import annotations

import statistics
from typing import Callable


def stamped_passes(launch: Callable[[], None], stream: int, passes: int, warm: int = 20) -> list[dict]:
    """Run ``warm`` unstamped then ``passes`` stamped launches back to back on
    ``stream`` (stamp, launch, stamp, launch, ..., stamp; no host sync in
    between) and return, per pass, its shader cycles, wall microseconds and
    mean shader clock (MHz)."""
    import torch

    from .. import hip

    H = hip()
    K = H.clock_stamp_slots()
    khz = H.wall_clock_rate_khz()
    stamps = torch.zeros(3 * K * (passes + 1), dtype=torch.int64, device="cuda")
    sb = 3 * K * 8  # bytes per stamp
    for _ in range(warm):
        launch()
    for i in range(passes):
        H.clock_stamp(stamps.data_ptr() + sb * i, stream)
        launch()
    H.clock_stamp(stamps.data_ptr() + sb * passes, stream)
    torch.cuda.synchronize()
    v = stamps.cpu().view(passes + 1, K, 3).tolist()
    out = []
    for i in range(passes):
        d0 = {int(x): (c, t) for x, c, t in v[i]}
        d1 = {int(x): (c, t) for x, c, t in v[i + 1]}
        span_us = (max(t for _, t in d1.values()) - min(t for _, t in d0.values())) / (khz / 1e3)
        per_xcd: dict[int, list[float]] = {}
        for x in set(d0) & set(d1):
            if d1[x][1] > d0[x][1]:
                per_xcd.setdefault(x >> 16, []).append((d1[x][0] - d0[x][0]) / ((d1[x][1] - d0[x][1]) / (khz / 1e3)))
        xcd_mhz = sorted(statistics.median(v) for v in per_xcd.values())
        clock = statistics.median([m for v in per_xcd.values() for m in v]) if per_xcd else 0.0
        slow = xcd_mhz[0] if xcd_mhz else 0.0
        out.append({"cycles": span_us * slow, "cycles_median_clock": span_us * clock, "us": span_us, "mhz": clock,
                    "mhz_slowest_xcd": slow, "xcd_spread": (xcd_mhz[-1] / slow - 1.0) if slow else 0.0,
                    "xcd_mhz": {k: statistics.median(v) for k, v in sorted(per_xcd.items())}})
    return out


def pass_cycles(launch: Callable[[], None], stream: int, passes: int = 24, warm: int = 20) -> dict:
    """Median shader cycles per pass over ``passes`` stamped passes, with the
    spread (min / max) and the median wall time and clock."""
    rows = stamped_passes(launch, stream, passes, warm)
    cyc = sorted(r["cycles"] for r in rows)
    med = statistics.median
    return {"cycles": med(cyc), "cycles_min": cyc[0], "cycles_max": cyc[-1],
            "cycles_median_clock": med(r["cycles_median_clock"] for r in rows),
            "us": med(r["us"] for r in rows), "mhz": med(r["mhz"] for r in rows),
            "mhz_slowest_xcd": med(r["mhz_slowest_xcd"] for r in rows),
            "xcd_spread": med(r["xcd_spread"] for r in rows), "passes": passes}
