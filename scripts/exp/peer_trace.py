"""Kernel timeline of the N > 1 window, rehearsed on one GPU: the 8-GPU tile
through RCCL loopback in the peers' schedule (MXS_PEER_SCHEDULE=1: prime
exchange, then a bare pass). Runs --reps 20-step windows separated by idle gaps,
so `scripts/exp/rocpd_timeline.py` can cut the kernel trace into windows.

    rocprofv3 --kernel-trace -d OUT -o trace -- python3 scripts/exp/peer_trace.py
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

os.environ["MXS_PEER_SCHEDULE"] = "1"  # read by the solver's constructor
from cuda_mpi_scratch_amd.models.stencil2d import Stencil2D, StencilConfig  # noqa: E402
from cuda_mpi_scratch_amd.parallel import init  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--tile", default="16384x8192")
p.add_argument("--k", type=int, default=20)
p.add_argument("--reps", type=int, default=12)
p.add_argument("--halo-last", action="store_true", help="the interior-first schedule instead of the serial one")
a = p.parse_args()
w, h = (int(x) for x in a.tile.split("x"))
ctx = init(backend="gloo", device="cuda")
st = Stencil2D(StencilConfig(global_width=w, global_height=h, dims="1x1", dtype="f32", loopback=True,
                             frame_overlap=False, halo_last=a.halo_last), ctx)
st.run(5)
st.prepare(a.k)
st.warm(a.k, 0.1)
st.synchronize()
for i in range(a.reps):
    torch.cuda.synchronize()
    time.sleep(0.003)  # idle gap: the timeline script splits windows here
    t0 = time.perf_counter()
    st.run(a.k)
    st.synchronize()
    print(f"window {i}: {(time.perf_counter() - t0) * 1e3:.4f} ms, exchanges {st.solver.last_run_exchanges()}",
          flush=True)
ctx.destroy()
