"""Clock-independent cost of a kernel launch: shader cycles per pass.

The stencil passes are VALU-bound and the chip's shader clock follows its power
management (1.5-2.05 GHz under this load, docs/PERF.md "The clock, measured"),
so a pass's wall time moves by +-10% from box to box and run to run while its
cost in shader cycles stays within ~2.5%. Cycles are measured from two
``hip().clock_stamp`` launches around each pass (512 one-wave workgroups; each
records its CU's shader-clock counter ``s_memtime`` and the global 100 MHz wall
clock): the pass's wall span is the last "after" stamp minus the first "before"
stamp, its mean clock the median over the CUs seen in both stamps of
(counter delta / wall delta), and cycles = span x clock.

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
        mhz = [(d1[x][0] - d0[x][0]) / ((d1[x][1] - d0[x][1]) / (khz / 1e3))
               for x in set(d0) & set(d1) if d1[x][1] > d0[x][1]]
        clock = statistics.median(mhz) if mhz else 0.0
        out.append({"cycles": span_us * clock, "us": span_us, "mhz": clock})
    return out


def pass_cycles(launch: Callable[[], None], stream: int, passes: int = 24, warm: int = 20) -> dict:
    """Median shader cycles per pass over ``passes`` stamped passes, with the
    spread (min / max) and the median wall time and clock."""
    rows = stamped_passes(launch, stream, passes, warm)
    cyc = sorted(r["cycles"] for r in rows)
    return {"cycles": statistics.median(cyc), "cycles_min": cyc[0], "cycles_max": cyc[-1],
            "us": statistics.median(r["us"] for r in rows), "mhz": statistics.median(r["mhz"] for r in rows),
            "passes": passes}
