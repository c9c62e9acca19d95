"""Per-pass time over a long run (run under rocprofv3 --kernel-trace): does a
pass slow down as the field evolves (data) or stay flat after the clock settles?

Phases on 8192^2 fp32 (sum form, S = 20), each separated by a 50 ms host sleep:
  A: 200 state-preserving passes (warm: cur -> nxt, the field never changes)
  B: run(4800) = 240 passes that advance the field
  C: 200 state-preserving passes again (on the evolved field)
  D: fresh random field (new Stencil2D), run(4800)"""
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))))
from cuda_mpi_scratch_amd.models.stencil2d import Stencil2D, StencilConfig  # noqa: E402


def main() -> int:
    dtype = sys.argv[1] if len(sys.argv) > 1 else "f32"
    cfg = StencilConfig(global_width=8192, global_height=8192, dims="1x1", dtype=dtype)
    st = Stencil2D(cfg)
    S = st.time_block
    st.run(48)
    st.prepare(S)
    st.synchronize()
    for phase in "ABC":
        time.sleep(0.05)
        t0 = time.perf_counter()
        if phase == "B":
            st.run(240 * S)
        else:
            st.solver.warm(S, 200)
        st.synchronize()
        torch.cuda.synchronize()
        print(phase, round((time.perf_counter() - t0) * 1e3, 2), "ms", flush=True)
    del st
    time.sleep(0.05)
    st = Stencil2D(StencilConfig(global_width=8192, global_height=8192, dims="1x1", dtype=dtype, seed=7))
    st.run(S)
    st.synchronize()
    t0 = time.perf_counter()
    st.run(240 * S)
    st.synchronize()
    print("D", round((time.perf_counter() - t0) * 1e3, 2), "ms", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
