"""Clock-normalised performance regression tests.

The rate floors of tests/test_gpu_headline.py (Gcells/s) must leave room for the
chip's clock, which moves the same pass by +-10% (docs/PERF.md: 1.5-2.05 GHz),
so a 25% slower kernel still passed them. These tests hold the passes'
cost in SHADER CYCLES (cuda_mpi_scratch_amd/utils/cycles.py: clock stamps
around each pass, CU-matched) to a budget of about 5% over the measured
counts, which does not depend on the clock a box happens to run at:

  * the headline pass: 32768^2 fp32, 20 levels, periodic wrap, sum form
    (bench.py's N = 1 window);
  * BASELINE config 2: 8192^2 fp32 at its auto time block, wrap, sum form;
  * fp64: 8192^2, 16 levels (the fp64 pipeline), wrap, sum form;
  * the 8-GPU rank tile: 16384 x 8192 fp32, 20 levels on the ghost-ring tile
    (no wrap: the N = 8 run's pass).

The budgets were measured on MI355X boxes (profiles/r06_cycles). A build that
adds ~10% VALU to the pass body fails them (checked by hand: profiles/r06_cycles).
"""
import json

import pytest
import torch

from cuda_mpi_scratch_amd import core, hip
from cuda_mpi_scratch_amd.ops import fill_random
from cuda_mpi_scratch_amd.utils.cycles import pass_cycles

pytestmark = pytest.mark.gpu

# name: (width, height, dtype, levels (0: auto_time_block), wrap, budget). The VALU-bound
# fp32 passes are held in k shader cycles per pass at the slowest XCD's clock (two boxes:
# 3647 / 3652, 277.3 / 277.8, 505.6 / 506.1; budgets +5%). The fp64 pass is HBM-bound
# (S = 16: 1 B per cell-level against a 19-slot VALU body): its cycles follow the clock
# (433-477 k at 1.82-2.0 GHz) while its time does not (242-245 us), so it is held in us.
CASES = {
    "headline_32768sq_f32": (32768, 32768, "f32", 20, True, ("kcycles", 3830.0)),
    "config2_8192sq_f32": (8192, 8192, "f32", 0, True, ("kcycles", 291.0)),
    "fp64_8192sq": (8192, 8192, "f64", 16, True, ("us", 257.0)),
    "tile8_16384x8192_f32": (16384, 8192, "f32", 20, False, ("kcycles", 531.0)),
}


@pytest.mark.parametrize("name", list(CASES))
def test_pass_cycles_within_budget(gpu, name):
    w, h, dtype, S, wrap, budget = CASES[name]
    H, C = hip(), core()
    if S == 0:
        S = H.auto_time_block(w, h, dtype, True)
    tdt = torch.float32 if dtype == "f32" else torch.float64
    g = C.TileGeom.aligned(w, h, S, S, tdt.itemsize)
    a = torch.zeros(g.alloc_elems(), dtype=tdt, device=gpu)
    b = torch.zeros_like(a)
    fill_random(a, g, 0, 0, w, 4321)  # random data: zeros would raise the clock, not change the cycles
    fill_random(b, g, 0, 0, w, 4322)
    s = torch.cuda.current_stream().cuda_stream
    bufs = [a, b]

    def launch():
        H.stencil5_tb(bufs[0].data_ptr(), bufs[1].data_ptr(), g, S, 0, w, 0, h, 0.2, 0.2, wrap, dtype, s, "auto",
                      True)
        bufs.reverse()  # ping-pong as the solver does (re-reading one input would stay in the Infinity Cache)

    r = pass_cycles(launch, s, passes=24, warm=40 if w * h >= 1 << 28 else 200)
    kernel = H.last_stencil_dispatch()
    rec = {"case": name, "S": S, "kernel": kernel, "lag1": bool(H.last_pipe_lag1()),
           "kcycles": round(r["cycles"] / 1e3, 1), "kcycles_min": round(r["cycles_min"] / 1e3, 1),
           "kcycles_max": round(r["cycles_max"] / 1e3, 1),
           "kcycles_median_clock": round(r["cycles_median_clock"] / 1e3, 1), "us": round(r["us"], 1),
           "mhz": round(r["mhz"]), "mhz_slowest_xcd": round(r["mhz_slowest_xcd"]),
           "xcd_spread": round(r["xcd_spread"], 3), "budget": budget}
    print(json.dumps(rec))
    assert kernel.startswith("stream_pipe_sum"), kernel
    unit, limit = budget
    got = r["cycles"] / 1e3 if unit == "kcycles" else r["us"]
    assert got <= limit, rec
