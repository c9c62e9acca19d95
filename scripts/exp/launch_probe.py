"""Host cost of one timed window's enqueue on the fused 8-GPU tile and the 1-GPU
tile: Stencil2D.run(20) (Python -> solver.run -> one pipeline launch), the bare
pybind stencil5_tb launch of the same pass, and an empty torch kernel, each
timed on the host from call to return (the GPU drained before each call), and
the GPU's idle gap from the call to the kernel's start (an event recorded just
before the call on the same stream is not possible from Python for the solver's
own stream, so the gap is estimated as window - event-timed pass).

usage: python scripts/exp/launch_probe.py [REPS]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from cuda_mpi_scratch_amd import hip  # noqa: E402
from cuda_mpi_scratch_amd.models.stencil2d import Stencil2D, StencilConfig  # noqa: E402


def med(v):
    v = sorted(v)
    return round(v[len(v) // 2], 2)


def main() -> int:
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    H = hip()
    out = {}
    for tile in ("16384x8192", "32768x32768"):
        w, h = (int(x) for x in tile.split("x"))
        st = Stencil2D(StencilConfig(global_width=w, global_height=h, dims="1x1", dtype="f32", seed=3))
        st.run(20)
        st.prepare(20)
        st.synchronize()
        a = st.current()
        b = st.b if a.data_ptr() == st.a.data_ptr() else st.a
        s = torch.cuda.current_stream()
        t_run, t_launch, t_empty, t_window = [], [], [], []
        x = torch.zeros(1, device="cuda")
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            st.run(20)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            t_run.append((t1 - t0) * 1e6)
            t_window.append((t2 - t0) * 1e6)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            H.stencil5_tb(a.data_ptr(), b.data_ptr(), st.geom, 20, 0, w, 0, h, 0.2, 0.2, True, stream=s.cuda_stream)
            t1 = time.perf_counter()
            t_launch.append((t1 - t0) * 1e6)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            x.add_(1.0)
            t1 = time.perf_counter()
            t_empty.append((t1 - t0) * 1e6)
        out[tile] = {"run20_host_us": med(t_run), "pybind_stencil5_tb_host_us": med(t_launch),
                     "torch_add_host_us": med(t_empty), "run20_window_us": med(t_window)}
        print(json.dumps({tile: out[tile]}), flush=True)
        del st
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
