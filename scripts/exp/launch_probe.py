"""Where the fixed per-window host cost goes (round-4 verdict, Weak 6). One
process, interleaved rounds of four windows, each from a drained device and
timed on the host clock like the bench's window (t0, enqueue, device sync):

  empty    one spin_delay(0) launch (a one-wave kernel that returns at once):
           the floor of launch + completion + sync on this box;
  fused    run(20) of the fused-periodic 8-GPU tile (one 20-level pass);
  pass     the same pass launched directly (stencil5_tb, no solver);
  span     the fused pass's GPU time alone (events around it, median).

Prints per-kind medians of the window and of the enqueue (t0 to the launch
call's return); fused - span is the window's fixed cost, empty is the part of
it any single launch pays.

usage: python scripts/exp/launch_probe.py [TILE] [ROUNDS]"""
import json
import statistics
import sys
import time

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__)))))

import torch  # noqa: E402

from cuda_mpi_scratch_amd import hip  # noqa: E402
from cuda_mpi_scratch_amd.models.stencil2d import Stencil2D, StencilConfig  # noqa: E402


def main() -> int:
    tile = sys.argv[1] if len(sys.argv) > 1 else "16384x8192"
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    w, h = (int(x) for x in tile.split("x"))
    H = hip()
    st = Stencil2D(StencilConfig(global_width=w, global_height=h, dims="1x1", dtype="f32", seed=5))
    st.run(20)
    st.prepare(20)
    st.warm(20, 0.2)
    st.synchronize()
    s = torch.cuda.current_stream()
    a, b = st.a, st.b
    g = st.geom
    rows = {"empty": ([], []), "fused": ([], []), "pass": ([], []), "span": ([], [])}

    def window(kind, fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        tr = time.perf_counter()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        rows[kind][0].append((t1 - t0) * 1e6)
        rows[kind][1].append((tr - t0) * 1e6)

    def direct_pass():
        H.stencil5_tb(a.data_ptr(), b.data_ptr(), g, 20, 0, w, 0, h, 0.2, 0.2, True, dtype="f32",
                      stream=s.cuda_stream, variant="auto", sum_form=True)

    for _ in range(rounds):
        window("empty", lambda: H.spin_delay(0.0, s.cuda_stream))
        window("fused", lambda: st.run(20))
        window("pass", direct_pass)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(s)
        direct_pass()
        e1.record(s)
        torch.cuda.synchronize()
        rows["span"][0].append(e0.elapsed_time(e1) * 1e3)
        rows["span"][1].append(0.0)
    out = {"tile": tile, "rounds": rounds, "solver_stream_is_torch_current": False}
    for k, (win, enq) in rows.items():
        out[k] = {"window_us_median": round(statistics.median(win), 1), "window_us_p10": round(sorted(win)[len(win) // 10], 1),
                  "enqueue_us_median": round(statistics.median(enq), 1)}
    out["fixed_cost_us"] = round(out["fused"]["window_us_median"] - out["span"]["window_us_median"], 1)
    print(json.dumps(out), flush=True)
    # B. The bench's shape: warm() (~200 ms of passes), drain, then three
    # windows in a row; with --pre, an empty kernel + sync just before the
    # first window's t0 (outside it). Is the first window after the burst the
    # slow one, and does a pre-launch change that?
    seq = {"after_warm": [[], [], []], "after_warm_pre": [[], [], []]}
    for r in range(max(4, rounds // 6)):
        for kind in seq:
            st.warm(20, 0.2)
            st.synchronize()
            torch.cuda.synchronize()
            for i in range(3):
                if kind.endswith("_pre") and i == 0:
                    H.spin_delay(0.0, s.cuda_stream)
                    torch.cuda.synchronize()
                t0 = time.perf_counter()
                st.run(20)
                torch.cuda.synchronize()
                seq[kind][i].append((time.perf_counter() - t0) * 1e6)
    print(json.dumps({k: [round(statistics.median(v), 1) for v in vs] for k, vs in seq.items()}
                     | {"raw_" + k: [[round(x, 1) for x in v] for v in vs] for k, vs in seq.items()}), flush=True)
    # C. The same after-warm sequence with events on the solver's own stream
    # around each run(20): is the first window's extra time GPU time (the pass
    # runs slower) or host time (launch / completion)?
    ms = torch.cuda.ExternalStream(st.solver.main_stream())
    walls, spans = [[], [], []], [[], [], []]
    for r in range(max(4, rounds // 6)):
        st.warm(20, 0.2)
        st.synchronize()
        torch.cuda.synchronize()
        for i in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record(ms)
            st.run(20)
            e1.record(ms)
            torch.cuda.synchronize()
            walls[i].append((time.perf_counter() - t0) * 1e6)
            spans[i].append(e0.elapsed_time(e1) * 1e3)
    # D. What ends the post-burst transient? After warm(): nothing, an empty
    # launch + sync, one more warm pass + sync (the second-window state), or a
    # 1 ms sleep; then one event-bracketed window.
    variants = {"none": lambda: None,
                "empty": lambda: (H.spin_delay(0.0, s.cuda_stream), torch.cuda.synchronize()),
                "one_pass": lambda: (st.warm(20, 1e-9), st.synchronize()),
                "sleep1ms": lambda: time.sleep(0.001)}
    dres = {k: ([], []) for k in variants}
    for r in range(max(6, rounds // 5)):
        for k, act in variants.items():
            st.warm(20, 0.2)
            st.synchronize()
            torch.cuda.synchronize()
            act()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record(ms)
            st.run(20)
            e1.record(ms)
            torch.cuda.synchronize()
            dres[k][0].append((time.perf_counter() - t0) * 1e6)
            dres[k][1].append(e0.elapsed_time(e1) * 1e3)
    print(json.dumps({"after_warm_variants": {k: {"wall_us": round(statistics.median(w), 1),
                                                  "span_us": round(statistics.median(sp), 1),
                                                  "host_us": round(statistics.median([a - b for a, b in zip(w, sp)]), 1)}
                                              for k, (w, sp) in dres.items()}}), flush=True)
    print(json.dumps({"after_warm_events": {"wall_us": [round(statistics.median(v), 1) for v in walls],
                                            "span_us": [round(statistics.median(v), 1) for v in spans],
                                            "raw_span_us": [[round(x, 1) for x in v] for v in spans]}}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
