"""Host overhead of the driver's timed window on one GPU (run under rocprofv3
--kernel-trace to get each window's kernel time): the bench's sequence
(run -> solver.synchronize -> torch.cuda.synchronize) against a window that
spins on hipStreamQuery of the solver's main stream instead of blocking."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cuda_mpi_scratch_amd.models.stencil2d import Stencil2D, StencilConfig  # noqa: E402


def main() -> int:
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
    st = Stencil2D(StencilConfig(global_width=n, global_height=n, dims="1x1", dtype="f32"))
    stream = torch.cuda.ExternalStream(st.solver.main_stream())
    st.run(5)
    st.prepare(20)
    st.warm(20, 0.2)
    st.synchronize()
    torch.cuda.synchronize()
    for rep in range(6):
        for mode in ("block", "spin"):
            st.synchronize()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            st.run(20)
            t_launch = time.perf_counter()
            if mode == "block":
                st.synchronize()
                torch.cuda.synchronize()
            else:
                while not stream.query():
                    pass
            t1 = time.perf_counter()
            print(f"{mode} window_us {1e6 * (t1 - t0):.1f} launch_us {1e6 * (t_launch - t0):.1f}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
