"""Outer-set size of the interior-first opening, measured: the 8-GPU tile's
20-step window in the peers' schedule with MXS_HALO_LAST_WGS = each value
(the schedule is built at prepare(), which reads it), interleaved window by
window, against the serial opening.

    python scripts/exp/halo_last_wgs.py [--tile 16384x8192] [--wgs 24 32 40 48] [--reps 40]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

os.environ["MXS_PEER_SCHEDULE"] = "1"
from cuda_mpi_scratch_amd.models.stencil2d import Stencil2D, StencilConfig  # noqa: E402
from cuda_mpi_scratch_amd.parallel import init  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--tile", default="16384x8192")
p.add_argument("--wgs", type=int, nargs="+", default=[24, 32, 40, 48])
p.add_argument("--min", type=int, default=8)
p.add_argument("--reps", type=int, default=40)
a = p.parse_args()
w, h = (int(x) for x in a.tile.split("x"))
ctx = init(backend="gloo", device="cuda")
sts = {"serial": Stencil2D(StencilConfig(global_width=w, global_height=h, dims="1x1", loopback=True,
                                         frame_overlap=False), ctx)}
sts["serial"].run(5)
sts["serial"].prepare(20)
os.environ["MXS_HALO_LAST_MIN_WGS"] = str(a.min)
for m in a.wgs:
    os.environ["MXS_HALO_LAST_WGS"] = str(m)
    st = Stencil2D(StencilConfig(global_width=w, global_height=h, dims="1x1", loopback=True, frame_overlap=False,
                                 halo_last=True), ctx)
    st.run(5)
    st.prepare(20)
    sts[f"halo_last_{m}"] = st
for st in sts.values():
    st.warm(20, 0.05)
    st.synchronize()
ms = {n: [] for n in sts}
for i in range(a.reps):
    for n, st in sts.items():
        st.synchronize()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st.run(20)
        st.synchronize()
        ms[n].append((time.perf_counter() - t0) * 1e3)
for n, v in ms.items():
    v.sort()
    print(json.dumps({"tile": a.tile, "schedule": n, "median_ms": round(v[len(v) // 2], 4), "min_ms": round(v[0], 4),
                      "p90_ms": round(v[int(len(v) * 0.9)], 4)}), flush=True)
ctx.destroy()
