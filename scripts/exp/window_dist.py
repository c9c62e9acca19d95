"""Distribution of 20-step windows on the 8-GPU tile (16384 x 8192), timed the
way bench.py times one (barrier + sync, run(20), synchronize): fused vs RCCL
loopback, with and without the communication watchdog's polling wait."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from cuda_mpi_scratch_amd import hip  # noqa: E402
from cuda_mpi_scratch_amd.models.stencil2d import Stencil2D, StencilConfig  # noqa: E402
from cuda_mpi_scratch_amd.parallel import init  # noqa: E402

ctx = init(backend="gloo", device="cuda")
for loopback in (False, True):
    for timeout in (300.0, 0.0):
        if not loopback and timeout == 0.0:
            continue
        hip().set_comm_timeout(timeout)
        st = Stencil2D(StencilConfig(global_width=16384, global_height=8192, dims="1x1", dtype="f32",
                                     loopback=loopback), ctx)
        st.run(5)
        st.prepare(20)
        st.warm(20, 0.2)
        ms = []
        for i in range(40):
            st.synchronize()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            st.run(20)
            st.synchronize()
            torch.cuda.synchronize()
            ms.append((time.perf_counter() - t0) * 1e3)
            if i % 10 == 9:
                time.sleep(0.01)  # an idle gap, as between bench phases
        ms.sort()
        print(json.dumps({"loopback": loopback, "comm_timeout": timeout, "min_ms": round(ms[0], 4),
                          "median_ms": round(ms[len(ms) // 2], 4), "p90_ms": round(ms[int(len(ms) * 0.9)], 4),
                          "max_ms": round(ms[-1], 4)}), flush=True)
        del st
ctx.destroy()
