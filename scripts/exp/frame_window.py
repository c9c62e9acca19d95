"""Interleaved window timing on one GPU of the multi-GPU schedules for a
per-GPU tile (default the 8-GPU tile 16384 x 8192): fused periodic (no
exchange), RCCL loopback serial (exchange, then pass) and RCCL loopback
frame-first overlap with several comm-workgroup counts. Each window is timed
the way bench.py times one (sync, run(K), synchronize); configurations are
interleaved window by window so box-level clock drift hits them all alike.

    python scripts/exp/frame_window.py [--tile 16384x8192] [--k 20] [--reps 40]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from cuda_mpi_scratch_amd.models.stencil2d import Stencil2D, StencilConfig  # noqa: E402
from cuda_mpi_scratch_amd.parallel import init  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--tile", default="16384x8192")
p.add_argument("--k", type=int, nargs="+", default=[20, 240])
p.add_argument("--reps", type=int, default=40)
p.add_argument("--comm", type=int, nargs="+", default=[8, 0, 16])
p.add_argument("--frame-rows", type=int, default=0)
p.add_argument("--out", default=None)
a = p.parse_args()
w, h = (int(x) for x in a.tile.split("x"))
ctx = init(backend="gloo", device="cuda")
confs = {"fused": dict(), "serial": dict(loopback=True, graph_max_superstep_us=0),
         "serial_eager": dict(loopback=True, graph=False)}
for c in a.comm:
    confs[f"frame_c{c}"] = dict(loopback=True, frame_overlap=True, frame_comm_wgs=c, frame_rows=a.frame_rows)
sts = {name: Stencil2D(StencilConfig(global_width=w, global_height=h, dims="1x1", dtype="f32", **kw), ctx)
       for name, kw in confs.items()}
recs = []
for K in a.k:
    for st in sts.values():
        st.run(5)
        st.prepare(K)
        st.warm(K, 0.1)
        st.synchronize()
    ms = {n: [] for n in sts}
    reps = a.reps if K <= 40 else max(3, a.reps // 8)
    for i in range(reps):
        for n, st in sts.items():
            st.synchronize()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            st.run(K)
            st.synchronize()
            ms[n].append((time.perf_counter() - t0) * 1e3)
    for n, v in ms.items():
        v.sort()
        r = {"tile": a.tile, "K": K, "schedule": n, "reps": len(v), "min_ms": round(v[0], 4),
             "median_ms": round(v[len(v) // 2], 4), "p90_ms": round(v[int(len(v) * 0.9)], 4), "max_ms": round(v[-1], 4),
             "median_gcells_per_s": round(w * h * K / (v[len(v) // 2] * 1e-3) / 1e9, 1)}
        if n.startswith("frame"):
            s = sts[n].solver.frame_schedule(sts[n].time_block)
            if s:
                r.update(frame_cost=s["frame_cost"], bulk_cost=s["bulk_cost"], signals=s["signals"])
        recs.append(r)
        print(json.dumps(r), flush=True)
if a.out:
    with open(a.out, "w") as f:
        for r in recs:
            f.write(json.dumps(r) + "\n")
ctx.destroy()
