"""Where a short timed window's time goes (bench.py's timed_run around run(K)):
host time of run() (launch path), of the solver's synchronize(), of the
closing torch.cuda.synchronize(), against the GPU time between events recorded
on the solver's main stream right before and after run(K)."""
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
p.add_argument("--global", dest="g", default="8192x8192")
p.add_argument("--k", type=int, default=20)
p.add_argument("--reps", type=int, default=30)
p.add_argument("--loopback", action="store_true")
p.add_argument("--graph", choices=["auto", "on", "off"], default="auto")
a = p.parse_args()
w, h = (int(x) for x in a.g.split("x"))
ctx = init(backend="gloo", device="cuda")
kw = {}
if a.graph == "on":
    kw["graph_max_superstep_us"] = 0
elif a.graph == "off":
    kw["graph"] = False
st = Stencil2D(StencilConfig(global_width=w, global_height=h, dims="1x1", dtype="f32", loopback=a.loopback, **kw), ctx)
st.run(5)
st.prepare(a.k)
st.warm(a.k, 0.2)
st.synchronize()
ms = torch.cuda.ExternalStream(st.solver.main_stream())
rec = {k: [] for k in ("run_us", "sync_us", "torch_sync_us", "window_us", "gpu_us")}
for i in range(a.reps):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(ms)
    st.run(a.k)
    e1.record(ms)
    t1 = time.perf_counter()
    st.synchronize()
    t2 = time.perf_counter()
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    rec["run_us"].append((t1 - t0) * 1e6)
    rec["sync_us"].append((t2 - t1) * 1e6)
    rec["torch_sync_us"].append((t3 - t2) * 1e6)
    rec["window_us"].append((t3 - t0) * 1e6)
    rec["gpu_us"].append(e0.elapsed_time(e1) * 1e3)
out = {"global": a.g, "K": a.k, "loopback": a.loopback, "graph": st.graph_status()}
for k, v in rec.items():
    v.sort()
    out[k] = round(v[len(v) // 2], 1)
print(json.dumps(out), flush=True)
ctx.destroy()
