"""The opening decision on the 8-GPU tile through RCCL loopback in the peers'
schedule: prepare()'s agreed numbers (paired ratio, notch, reason) for a few
fresh solvers, and event-timed replicas (profile_window) of the serial and the
interior-first openings, interleaved, as the bench records them.

usage: python scripts/exp/opening_probe.py [TILE] [SOLVERS] [REPLICAS] [WIRE_US]
(WIRE_US: rehearsed wire time after each RCCL transfer, SolverConfig::wire_delay_us)"""
import json
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__)))))

import torch  # noqa: E402

from cuda_mpi_scratch_amd.models.stencil2d import Stencil2D, StencilConfig  # noqa: E402


def main() -> int:
    tile = sys.argv[1] if len(sys.argv) > 1 else "16384x8192"
    solvers = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    w, h = (int(x) for x in tile.split("x"))
    kw = dict(global_width=w, global_height=h, dims="1x1", dtype="f32", backend="rccl", loopback=True,
              rehearse_peers=True, seed=5, wire_delay_us=float(sys.argv[4]) if len(sys.argv) > 4 else 0.0)
    for i in range(solvers):
        st = Stencil2D(StencilConfig(**kw))
        st.run(20)
        st.prepare(20)
        print(json.dumps({"solver": i, **st.solver.schedule_times()}), flush=True)
        del st
        torch.cuda.empty_cache()
    sts = {o: Stencil2D(StencilConfig(opening=o, **kw)) for o in ("serial", "interior-first")}
    for st in sts.values():
        st.run(20)
        st.prepare(20)
        st.warm(20, 0.2)
    reps_ = {o: [] for o in sts}
    for _ in range(reps):
        for o, st in sts.items():
            reps_[o].append(st.profile_window(20))
    spans = {o: [p["gpu_span_us"] for p in v] for o, v in reps_.items()}
    for o, v in reps_.items():
        v = sorted(v, key=lambda p: p["gpu_span_us"])
        med = v[len(v) // 2]
        print(json.dumps({"opening": o, "gpu_span_us_median": med["gpu_span_us"], "min": v[0]["gpu_span_us"],
                          "max": v[-1]["gpu_span_us"], "median_phases": med["phases_us"],
                          "outer_wgs": sts[o].solver.schedule_times()["outer_wgs"]}))
    ratio = sorted(a / b for a, b in zip(spans["interior-first"], spans["serial"]))
    print(json.dumps({"paired_ratio_median": round(ratio[len(ratio) // 2], 4), "min": round(ratio[0], 4),
                      "max": round(ratio[-1], 4)}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
