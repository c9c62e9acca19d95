"""Fused halo pack, measured in one process on the 8-GPU tile through RCCL
loopback (peers' schedule): (1) the bare 20-level pass alone, event-timed, with
and without the pack epilogue (the pass's own cost of the fusion); (2)
interleaved event-timed replicas of the window's opening super-step
(profile_window) for the serial and interior-first openings, fused pack on and
off.

usage: python scripts/exp/pack_probe.py [TILE] [REPS]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from cuda_mpi_scratch_amd import core, hip  # noqa: E402
from cuda_mpi_scratch_amd.models.stencil2d import Stencil2D, StencilConfig  # noqa: E402


def med(v):
    v = sorted(v)
    return round(v[len(v) // 2], 1)


def main() -> int:
    tile = sys.argv[1] if len(sys.argv) > 1 else "16384x8192"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    w, h = (int(x) for x in tile.split("x"))
    kw = dict(global_width=w, global_height=h, dims="1x1", dtype="f32", backend="rccl", loopback=True,
              rehearse_peers=True, seed=5, time_block=20)
    H = hip()
    # (1) the bare pass, cur -> scratch, with and without the epilogue.
    st = Stencil2D(StencilConfig(**kw))
    st.run(20)
    st.synchronize()
    g, s = st.geom, torch.cuda.current_stream()
    plan = core().make_halo_plan(st.decomp.topo, 0, g, True, True)
    wins = core().send_windows(plan)
    send = torch.empty(plan.send_elems, dtype=torch.float32, device="cuda")
    a = st.current()
    b = st.b if a.data_ptr() == st.a.data_ptr() else st.a
    times = {"pass": [], "pass+pack": []}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    def bare():
        H.stencil5_tb(a.data_ptr(), b.data_ptr(), g, 20, 0, w, 0, h, 0.2, 0.2, False, stream=s.cuda_stream)

    def packed():
        assert H.stencil5_tb_packed(a.data_ptr(), b.data_ptr(), g, 20, 0.2, 0.2, send.data_ptr(), wins,
                                    stream=s.cuda_stream)

    for _ in range(3):
        bare()
        packed()
    for r in range(reps):
        for name in times:
            torch.cuda.synchronize()
            e0.record(s)
            bare() if name == "pass" else packed()
            e1.record(s)
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) * 1e3)
    print(json.dumps({"bare_pass_us": {k: med(v) for k, v in times.items()},
                      "min": {k: round(min(v), 1) for k, v in times.items()}}), flush=True)
    del st
    torch.cuda.empty_cache()
    # (2) replicas of the window's opening.
    sts = {}
    for opening in ("serial", "interior-first"):
        for fp in (True, False):
            x = Stencil2D(StencilConfig(opening=opening, fused_pack=fp, **kw))
            x.run(20)
            x.prepare(20)
            x.warm(20, 0.1)
            sts[(opening, fp)] = x
    spans = {k: [] for k in sts}
    for _ in range(reps):
        for k, x in sts.items():
            spans[k].append(x.profile_window(20))
    for (opening, fp), v in spans.items():
        v = sorted(v, key=lambda p: p["gpu_span_us"])
        print(json.dumps({"opening": opening, "fused_pack": fp, "gpu_span_us": [round(p["gpu_span_us"]) for p in v],
                          "median_phases": v[len(v) // 2]["phases_us"], "slowest_phases": v[-1]["phases_us"]}),
              flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
