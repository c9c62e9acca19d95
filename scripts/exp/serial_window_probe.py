"""Why the serial opening's window is slower after prepare() decided it (round 6).

In single-shot bench runs of the 8-GPU tile (profiles/r06_tiles) the processes
whose decision kept the serial opening ran their window at 0.308-0.356 ms with
40-80 us of host time in run(), while solvers built with opening = serial ran it
at 0.298-0.304 ms with 20-25 us, and the decision's own serial samples said
0.28-0.30 ms. This runs the bench's window shape (warm burst, a drained warm
pass, barrier, host-timed run(20) + syncs) several times in one process for:
  decided : opening auto with min_gain 0.5, so prepare() runs the whole decision
            (lead measurement, 20 paired rounds, three outer sets) and keeps serial;
  forced  : opening serial (no decision).
Per window: wall ms, run() host us, and (--trace) nothing else: run it under
rocprofv3 --hip-trace for the per-call breakdown.

usage: python scripts/exp/serial_window_probe.py MODE [--windows 6] [--tile 16384x8192]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from cuda_mpi_scratch_amd import hip  # noqa: E402
from cuda_mpi_scratch_amd.models.stencil2d import Stencil2D, StencilConfig  # noqa: E402
from cuda_mpi_scratch_amd.parallel import init as dist_init  # noqa: E402


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("mode", choices=["decided", "forced"])
    p.add_argument("--windows", type=int, default=6)
    p.add_argument("--tile", default="16384x8192")
    args = p.parse_args()
    ctx = dist_init(backend="nccl")
    hip().set_comm_timeout(120.0)
    w, h = (int(v) for v in args.tile.split("x"))
    kw = dict(opening="auto", min_gain=0.5) if args.mode == "decided" else dict(opening="serial")
    st = Stencil2D(StencilConfig(global_width=w, global_height=h, dims="1x1", dtype="f32", backend="rccl",
                                 loopback=True, rehearse_peers=True, **kw), ctx)
    st.run(5)
    st.prepare(20)
    rows = []
    for _ in range(args.windows):
        st.warm(20, 0.2, 1)
        st.synchronize()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st.run(20)
        tr = time.perf_counter()
        st.synchronize()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        rows.append({"window_ms": round((t1 - t0) * 1e3, 4), "run_host_us": round((tr - t0) * 1e6, 1),
                     "opening": st.solver.last_run_opening()})
    print(json.dumps({"mode": args.mode, "choice": st.solver.schedule_times()["opening"],
                      "window_ms_median": statistics.median(r["window_ms"] for r in rows),
                      "host_us_median": statistics.median(r["run_host_us"] for r in rows), "windows": rows}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
