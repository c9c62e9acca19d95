"""Does a solver whose prepare() measured interior-first as serialised (paired
ratio ~1.5) predict a serialised window? Repeatedly in one process: an auto
solver's decision (choice, median ratios per candidate), then at once a forced
interior-first and a forced serial solver on the same tile, each timing
WINDOWS bench-shaped windows (drained streams, run(20), the solver's polled
wait; host clock). If the decision says ~1.5 while the forced interior-first
windows stay near the serial ones, the decision's sampling creates the state.

usage: python scripts/exp/decision_vs_window.py [TILE] [ITERATIONS] [WINDOWS]"""
import json
import statistics
import sys
import time

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__)))))

import torch  # noqa: E402

from cuda_mpi_scratch_amd.models.stencil2d import Stencil2D, StencilConfig  # noqa: E402


def windows(st, n):
    out = []
    for _ in range(n):
        st.synchronize()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st.run(20)
        st.synchronize()
        out.append((time.perf_counter() - t0) * 1e6)
    return out


def main() -> int:
    tile = sys.argv[1] if len(sys.argv) > 1 else "16384x8192"
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    nwin = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    w, h = (int(x) for x in tile.split("x"))
    kw = dict(global_width=w, global_height=h, dims="1x1", dtype="f32", backend="rccl", loopback=True,
              rehearse_peers=True, seed=5)
    for it in range(iters):
        auto = Stencil2D(StencilConfig(**kw))
        auto.run(20)
        auto.prepare(20)
        t = auto.solver.schedule_times()
        cand = {wgs: round(statistics.median(r), 3) for wgs, r in t["local_candidate_ratios"]}
        del auto
        res = {}
        for o in ("interior-first", "serial"):
            st = Stencil2D(StencilConfig(opening=o, **kw))
            st.run(20)
            st.prepare(20)
            st.warm(20, 0.1)
            v = windows(st, nwin)
            res[o] = {"median_us": round(statistics.median(v), 1), "max_us": round(max(v), 1),
                      "note": st.solver.stream_note()}
            del st
        print(json.dumps({"iteration": it, "auto_choice": t["opening"], "auto_ratio": round(t["ratio"], 3),
                          "candidates": cand, "forced": res}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
