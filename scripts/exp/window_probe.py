"""Short timed windows after warm-up: does a 20-step window run at the
sustained rate, or does it pay a clock ramp? Prints per-window ms."""
import sys
import time

import torch

sys.path.insert(0, ".")
from cuda_mpi_scratch_amd.models.stencil2d import Stencil2D, StencilConfig  # noqa: E402

st = Stencil2D(StencilConfig(global_width=32768, global_height=32768, dims="1x1", dtype="f32"))
st.run(5)
st.prepare(20)
st.synchronize()
for i in range(6):
    t0 = time.perf_counter()
    st.run(20)
    st.synchronize()
    dt = time.perf_counter() - t0
    print(f"window {i}: {dt*1e3:.3f} ms  {st.cells_per_step*20/dt/1e9:.0f} Gcells/s", flush=True)
    if i == 2:
        time.sleep(0.5)  # idle gap: does the next window pay a ramp again?
t0 = time.perf_counter()
st.run(240)
st.synchronize()
dt = time.perf_counter() - t0
print(f"240 steps: {dt*1e3:.3f} ms  {st.cells_per_step*240/dt/1e9:.0f} Gcells/s")
