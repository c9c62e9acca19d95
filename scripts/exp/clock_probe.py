"""Is the pass-to-pass spread the chip's clock? (round-4 verdict, Weak 2a.)
Every 20-level pass on the 8-GPU tile is bracketed by clock stamps (512
one-wave workgroups over the CUs: the CU's id, its shader clock counter, which
follows DVFS, and the constant 100 MHz wall clock): the wall time of the pass
and the mean shader clock it ran at (median over the CUs seen in both stamps)
come from the same two stamps.

  A. continuous: PASSES passes back to back on one stream (no host sync), the
     GPU's clock under sustained load;
  B. windows: the bench's shape WINDOWS times: ~200 ms of back-to-back passes,
     a drain, a short host gap, then one stamped pass.

Prints per-pass (ms, MHz) series and their correlation; a pass time that
tracks 1 / clock names DVFS as the cause of the spread.

usage: python scripts/exp/clock_probe.py [TILE] [PASSES] [WINDOWS] [--wrap]"""
import json
import statistics
import sys
import time

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__)))))

import torch  # noqa: E402

from cuda_mpi_scratch_amd import core, hip  # noqa: E402
from cuda_mpi_scratch_amd.ops import fill_random  # noqa: E402


def corr(x, y):
    mx, my = statistics.fmean(x), statistics.fmean(y)
    sxy = sum((a - mx) * (b - my) for a, b in zip(x, y))
    sx = sum((a - mx) ** 2 for a in x) ** 0.5
    sy = sum((b - my) ** 2 for b in y) ** 0.5
    return sxy / (sx * sy) if sx and sy else 0.0


def main() -> int:
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    wrap = "--wrap" in sys.argv
    tile = args[0] if args else "16384x8192"
    passes = int(args[1]) if len(args) > 1 else 400
    windows = int(args[2]) if len(args) > 2 else 20
    w, h = (int(x) for x in tile.split("x"))
    S = 20
    H, C = hip(), core()
    khz = H.wall_clock_rate_khz()
    g = C.TileGeom.aligned(w, h, S, S, 4)
    n = g.alloc_elems()
    a = torch.zeros(n, dtype=torch.float32, device="cuda")
    b = torch.zeros(n, dtype=torch.float32, device="cuda")
    fill_random(a, g, 0, 0, w, 1234)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream().cuda_stream
    K = H.clock_stamp_slots()
    SB = 3 * K * 8  # bytes per stamp
    stamps = torch.zeros(3 * K * (passes + 1), dtype=torch.int64, device="cuda")

    def launch():
        H.stencil5_tb(a.data_ptr(), b.data_ptr(), g, S, 0, w, 0, h, 0.2, 0.2, wrap, dtype="f32", stream=s)

    def series(st, k):
        """(pass ms, median over the CUs seen in both stamps of the mean shader clock in MHz)."""
        v = st.cpu().view(-1, K, 3).tolist()
        out = []
        for i in range(k):
            d0 = {int(x): (c, t) for x, c, t in v[i]}
            d1 = {int(x): (c, t) for x, c, t in v[i + 1]}
            dt_us = (max(t for _, t in d1.values()) - min(t for _, t in d0.values())) / (khz / 1e3)
            mhz = []
            for x in set(d0) & set(d1):
                c0, t0 = d0[x]
                c1, t1 = d1[x]
                if t1 > t0:
                    mhz.append((c1 - c0) / ((t1 - t0) / (khz / 1e3)))
            out.append((dt_us / 1e3, statistics.median(mhz) if mhz else 0.0))
        return out

    # A. continuous
    for _ in range(20):
        launch()
    for i in range(passes):
        H.clock_stamp(stamps.data_ptr() + SB * i, s)
        launch()
    H.clock_stamp(stamps.data_ptr() + SB * passes, s)
    torch.cuda.synchronize()
    a_ser = series(stamps, passes)
    ms = [x[0] for x in a_ser]
    mhz = [x[1] for x in a_ser]
    rec_a = {"part": "continuous", "tile": tile, "wrap": wrap, "passes": passes,
             "ms_median": round(statistics.median(ms), 4), "ms_min": round(min(ms), 4), "ms_max": round(max(ms), 4),
             "mhz_median": round(statistics.median(mhz)), "mhz_min": round(min(mhz)), "mhz_max": round(max(mhz)),
             "corr_ms_inv_mhz": round(corr(ms, [1.0 / m for m in mhz]), 3),
             "series": [[round(x, 4), round(y)] for x, y in a_ser]}
    print(json.dumps(rec_a), flush=True)
    # B. windows in the bench's shape
    wst = torch.zeros(6 * K, dtype=torch.int64, device="cuda")
    rows = []
    for _ in range(windows):
        t_end = time.perf_counter() + 0.2
        while time.perf_counter() < t_end:  # ~200 ms of passes (warm())
            for _ in range(20):
                launch()
            torch.cuda.synchronize()
        time.sleep(0.0002)  # the drain + barrier gap before t0
        H.clock_stamp(wst.data_ptr(), s)
        launch()
        H.clock_stamp(wst.data_ptr() + SB, s)
        torch.cuda.synchronize()
        rows.append(series(wst, 1)[0])
    ms = [x[0] for x in rows]
    mhz = [x[1] for x in rows]
    print(json.dumps({"part": "windows", "windows": windows, "ms": [round(x, 4) for x in ms],
                      "mhz": [round(x) for x in mhz], "ms_median": round(statistics.median(ms), 4),
                      "mhz_median": round(statistics.median(mhz)),
                      "corr_ms_inv_mhz": round(corr(ms, [1.0 / m for m in mhz]), 3)}), flush=True)
    print(f"continuous: pass {rec_a['ms_min']}-{rec_a['ms_max']} ms (median {rec_a['ms_median']}), clock "
          f"{rec_a['mhz_min']}-{rec_a['mhz_max']} MHz, corr(ms, 1/MHz) {rec_a['corr_ms_inv_mhz']}", file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
