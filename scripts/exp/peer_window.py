"""The window an N > 1 run times, rehearsed on one GPU through RCCL loopback:
with peers every run() primes the ghost ring (a collective decision), so a
call of n super-steps used to issue n + 1 exchanges (prime + one after every
pass); it now ends on a bare pass (n exchanges); peer_halo_last: the interior-first schedule (each
super-step's own halo exchanged under its core chunks). MXS_PEER_SCHEDULE makes a
1-rank loopback solver follow the peers' schedule (1 = bare last pass, 2 = the
old n + 1 form). Interleaved window by window, timed as bench.py does.

    python scripts/exp/peer_window.py [--tile 16384x8192] [--k 20 240] [--reps 40] [--out F]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from cuda_mpi_scratch_amd.models.stencil2d import Stencil2D, StencilConfig  # noqa: E402
from cuda_mpi_scratch_amd.parallel import init  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--tile", default="16384x8192")
p.add_argument("--k", type=int, nargs="+", default=[20, 240])
p.add_argument("--reps", type=int, default=40)
p.add_argument("--out", default=None)
a = p.parse_args()
w, h = (int(x) for x in a.tile.split("x"))
ctx = init(backend="gloo", device="cuda")
confs = {"fused": ({}, None), "loopback_1rank": (dict(loopback=True, frame_overlap=False), None),
         "peer_n_plus_1": (dict(loopback=True, frame_overlap=False), "2"),
         "peer_bare_tail": (dict(loopback=True, frame_overlap=False), "1"),
         "peer_halo_last": (dict(loopback=True, frame_overlap=False, halo_last=True), "1")}
sts = {}
for name, (kw, env) in confs.items():
    if env is None:
        os.environ.pop("MXS_PEER_SCHEDULE", None)
    else:
        os.environ["MXS_PEER_SCHEDULE"] = env  # read by the solver's constructor
    sts[name] = Stencil2D(StencilConfig(global_width=w, global_height=h, dims="1x1", dtype="f32", **kw), ctx)
os.environ.pop("MXS_PEER_SCHEDULE", None)
recs = []
for K in a.k:
    for st in sts.values():
        st.run(5)
        st.prepare(K)
        st.warm(K, 0.1)
        st.synchronize()
    ms = {n: [] for n in sts}
    reps = a.reps if K <= 40 else max(3, a.reps // 8)
    for i in range(reps):
        for n, st in sts.items():
            st.synchronize()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            st.run(K)
            st.synchronize()
            ms[n].append((time.perf_counter() - t0) * 1e3)
    for n, v in ms.items():
        v.sort()
        st = sts[n]
        r = {"tile": a.tile, "K": K, "schedule": n, "reps": len(v), "min_ms": round(v[0], 4),
             "median_ms": round(v[len(v) // 2], 4), "p90_ms": round(v[int(len(v) * 0.9)], 4),
             "median_gcells_per_s": round(w * h * K / (v[len(v) // 2] * 1e-3) / 1e9, 1),
             "exchanges_per_call": int(st.solver.last_run_exchanges()),
             "super_steps": [list(b) for b in st.solver.last_run_blocks()],
             "runs_schedule": ("halo-last" if st.solver.halo_last(20) else
                               ("frame" if st.solver.frame_overlap(20) else "serial"))}
        recs.append(r)
        print(json.dumps(r), flush=True)
if a.out:
    with open(a.out, "w") as f:
        for r in recs:
            f.write(json.dumps(r) + "\n")
ctx.destroy()
