"""One process, one tile, the persistent stencil grid sized for 1/n of the GPU
(kernels::set_gpu_share): does a half-GPU grid reach half the full-GPU rate?
(Two co-located ranks run their 128-workgroup kernels 20-30% slower than one
256-workgroup kernel on the same total work; this separates the grid size
from the concurrency.)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import bench  # noqa: E402
from cuda_mpi_scratch_amd import hip  # noqa: E402
from cuda_mpi_scratch_amd.models.stencil2d import Stencil2D, StencilConfig  # noqa: E402
from cuda_mpi_scratch_amd.parallel import init  # noqa: E402

ctx = init(backend="gloo", device="cuda")
for shape in ("16384x4096", "16384x8192"):
    w, h = (int(v) for v in shape.split("x"))
    for share in (1, 2):
        st = Stencil2D(StencilConfig(global_width=w, global_height=h, dims="1x1", dtype="f32"), ctx)
        hip().set_gpu_share(share)
        dt = bench.timed_run(st, ctx, 240, 24, 0.2)
        print(json.dumps({"tile": shape, "gpu_share": share, "kernel": hip().last_stencil_dispatch(),
                          "gcells_s": round(st.cells_per_step * 240 / dt / 1e9, 1)}), flush=True)
        hip().set_gpu_share(1)
        del st
ctx.destroy()
