"""The two-stream tail (round-4 verdict, Weak 2b): ~2 in 125 interior-first
bench windows took 0.53-0.99 ms instead of ~0.30, their two launches running
one after the other. One process, many windows in the bench's shape (drained
streams, run(20), the solver's polled wait), each with host stamps; a window
past THRESHOLD x the median is a tail. Run it under `rocprofv3 --kernel-trace`
to get every kernel's queue, start and end: the tail windows' inner / outer
chunk launches then show whether they serialised on the GPU (same queue, or
the second one dispatched only after the first ended) or were late on the host.

usage: python scripts/exp/tail_probe.py [TILE] [WINDOWS] [--serial] [--wire US]
prints one JSON line per window (wall, enqueue, forks) and a summary line."""
import json
import statistics
import sys
import time

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__)))))

import torch  # noqa: E402

from cuda_mpi_scratch_amd.models.stencil2d import Stencil2D, StencilConfig  # noqa: E402


def main() -> int:
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    tile = args[0] if args else "16384x8192"
    windows = int(args[1]) if len(args) > 1 else 200
    opening = "serial" if "--serial" in sys.argv else "interior-first"
    wire = float(sys.argv[sys.argv.index("--wire") + 1]) if "--wire" in sys.argv else 0.0
    w, h = (int(x) for x in tile.split("x"))
    st = Stencil2D(StencilConfig(global_width=w, global_height=h, dims="1x1", dtype="f32", backend="rccl",
                                 loopback=True, rehearse_peers=True, opening=opening, seed=5, wire_delay_us=wire))
    st.run(5)
    st.prepare(20)
    st.warm(20, 0.2)
    st.synchronize()
    torch.cuda.synchronize()
    rows = []
    for i in range(windows):
        st.synchronize()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st.run(20)
        tr = time.perf_counter()
        st.synchronize()
        t1 = time.perf_counter()
        rows.append({"i": i, "wall_us": round((t1 - t0) * 1e6, 1), "enqueue_us": round((tr - t0) * 1e6, 1),
                     "forks": int(st.solver.last_run_forks()), "opening": st.solver.last_run_opening(),
                     "t_start_s": round(t0, 6)})
    med = statistics.median(r["wall_us"] for r in rows)
    for r in rows:
        r["tail"] = r["wall_us"] > 1.5 * med
        print(json.dumps(r))
    tails = [r["i"] for r in rows if r["tail"]]
    print(json.dumps({"summary": True, "tile": tile, "opening": opening, "wire_us": wire, "windows": windows,
                      "median_us": med, "p90_us": sorted(r["wall_us"] for r in rows)[int(0.9 * windows)],
                      "max_us": max(r["wall_us"] for r in rows), "tails": tails,
                      "side_stream": st.solver.stream_note()}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
