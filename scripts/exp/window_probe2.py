"""Clock-ramp check: short 20-step windows right after setup vs after a
sustained warm-up of the same kernel (state-preserving prepare() launches)."""
import sys
import time

sys.path.insert(0, ".")
from cuda_mpi_scratch_amd.models.stencil2d import Stencil2D, StencilConfig  # noqa: E402


def windows(st, tag, n=4):
    out = []
    for _ in range(n):
        t0 = time.perf_counter()
        st.run(20)
        st.synchronize()
        out.append((time.perf_counter() - t0) * 1e3)
    print(tag, " ".join(f"{x:.3f}" for x in out), "ms", flush=True)


st = Stencil2D(StencilConfig(global_width=32768, global_height=32768, dims="1x1", dtype="f32"))
st.run(5)
st.prepare(20)
st.synchronize()
windows(st, "cold      :")
for k in range(60):  # ~200 ms of the same kernel, scratch-only (prepare-style launches)
    st.solver.warm(20) if hasattr(st.solver, "warm") else st.run(20)
st.synchronize()
windows(st, "after heat:")
time.sleep(1.0)
windows(st, "after 1s idle:")
