"""The frame-first pass alone (no exchange) against the regular balanced pass on
the same ghost-ring tile, interleaved, hipEvent-timed per launch: isolates the
schedule's cost (extra fills of the frame chunks, early-exit comm workgroups)
from any interference with RCCL. Also reports whether both are bitwise equal."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from cuda_mpi_scratch_amd import core, hip  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--tile", default="16384x8192")
p.add_argument("--steps", type=int, default=20)
p.add_argument("--reps", type=int, default=20)
p.add_argument("--comm", type=int, nargs="+", default=[0, 4, 8, 16])
p.add_argument("--frame-rows", type=int, nargs="+", default=[0])
a = p.parse_args()
w, h = (int(x) for x in a.tile.split("x"))
S = a.steps
g = core().TileGeom.aligned(w, h, S, S, 4)
gen = torch.Generator(device="cuda").manual_seed(1)
src = torch.rand(g.alloc_elems(), generator=gen, device="cuda")
dst = torch.zeros_like(src)
ref = torch.zeros_like(src)
H = hip()
s = torch.cuda.current_stream()
H.stencil5_tb(src.data_ptr(), ref.data_ptr(), g, S, 0, w, 0, h, 0.2, 0.2, False, "f32", s.cuda_stream)
torch.cuda.synchronize()
variants = [("balanced", None, None), ("equal", None, None)]
for c in a.comm:
    for fr in a.frame_rows:
        variants.append((f"frame_c{c}_r{fr}", c, fr))
times = {v[0]: [] for v in variants}
info = {}
for rep in range(a.reps + 2):
    for name, c, fr in variants:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        if c is None:
            H.set_pipe_balanced(name == "balanced")
            H.stencil5_tb(src.data_ptr(), dst.data_ptr(), g, S, 0, w, 0, h, 0.2, 0.2, False, "f32", s.cuda_stream)
            e1.record()
            H.set_pipe_balanced(True)
        else:
            d = H.stencil5_frame_pass(src.data_ptr(), dst.data_ptr(), g, S, 0.2, 0.2, "f32", c, fr, s.cuda_stream)
            e1.record()
            info[name] = {k: v for k, v in d.items() if k != "kernel_us"}
        torch.cuda.synchronize()
        if rep >= 2:
            times[name].append(e0.elapsed_time(e1) * 1e3 if c is None else d["kernel_us"])
        if rep == 2:
            assert torch.equal(dst, ref), f"{name}: output differs from the regular pass"
for name, v in times.items():
    v.sort()
    r = {"tile": a.tile, "S": S, "variant": name, "median_us": round(v[len(v) // 2], 1), "min_us": round(v[0], 1),
         "max_us": round(v[-1], 1)}
    r.update(info.get(name, {}))
    print(json.dumps(r), flush=True)
