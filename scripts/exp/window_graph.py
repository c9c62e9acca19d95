"""20-step windows on the 8-GPU tile (16384 x 8192), timed as bench.py times one
(sync, run(20), synchronize): hipGraph launch vs direct kernel launches, fused
periodic vs RCCL loopback. Configurations interleave per round so clock and
box drift hit all of them alike."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from cuda_mpi_scratch_amd.models.stencil2d import Stencil2D, StencilConfig  # noqa: E402
from cuda_mpi_scratch_amd.parallel import init  # noqa: E402

ctx = init(backend="gloo", device="cuda")
gw, gh = (int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "16384x8192").split("x"))
cfgs = [(lb, g) for lb in (False, True) for g in (True, False)]
sts = {}
for lb, g in cfgs:
    st = Stencil2D(StencilConfig(global_width=gw, global_height=gh, dims="1x1", dtype="f32", loopback=lb, graph=g),
                   ctx)
    st.run(5)
    st.prepare(20)
    sts[(lb, g)] = st
ms = {c: [] for c in cfgs}
for rnd in range(12):
    for c in cfgs:
        st = sts[c]
        st.warm(20, 0.05)
        for _ in range(5):
            st.synchronize()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            st.run(20)
            st.synchronize()
            torch.cuda.synchronize()
            ms[c].append((time.perf_counter() - t0) * 1e3)
for (lb, g), v in ms.items():
    v.sort()
    print(json.dumps({"tile": f"{gw}x{gh}", "loopback": lb, "graph": g, "n": len(v), "min_ms": round(v[0], 4),
                      "median_ms": round(v[len(v) // 2], 4), "p90_ms": round(v[int(len(v) * 0.9)], 4)}), flush=True)
ctx.destroy()
