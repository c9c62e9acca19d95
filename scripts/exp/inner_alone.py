"""The interior-first pass's two launches timed alone against the one-launch pass (round 6).

In the bench's windows the interior-first opening's GPU span is 5-7% longer than
the fused pass on every rank tile, while the schedule's cost model
(chunk_schedule.hpp: rows + fills per workgroup, the outer set started `lead`
late) predicts 2-4%. This times, on a ghost-ring tile with no exchange, paired
per round after a warm burst (event-timed, medians over rounds):
  pass  : the one-launch pass (stencil5_tb, balanced shares on every CU);
  inner : the inner chunk list alone (blocks - outer workgroups);
  outer : the outer chunk list alone;
  both  : inner then outer on one stream.
and prints each over `pass` next to the model's inner_cost / serial_cost.

usage: python scripts/exp/inner_alone.py [--tiles 32768x16384:0.095,16384x16384:0.127,16384x8192:0.21] [--rounds 12]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from cuda_mpi_scratch_amd import core, hip  # noqa: E402


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--tiles", default="32768x16384:0.095,16384x16384:0.127,16384x8192:0.21")
    p.add_argument("--outer", default="0", help="comma list of outer workgroup counts (0: the model's)")
    p.add_argument("--rounds", type=int, default=12)
    args = p.parse_args()
    S = 20
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    for spec in args.tiles.split(","):
        tile, lf = spec.split(":")
        w, h = (int(v) for v in tile.split("x"))
        g = core().TileGeom.aligned(w, h, S, S, 4)
        src = torch.rand(g.alloc_elems(), device=dev, dtype=torch.float32)
        dst = torch.zeros_like(src)

        def tb():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            hip().stencil5_tb(src.data_ptr(), dst.data_ptr(), g, S, 0, w, 0, h, 0.2, 0.2, False, "f32", s, "auto", True)
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) * 1e3

        for outer in (int(v) for v in args.outer.split(",")):
            def chunk(part):
                d = hip().stencil5_chunk_pass(src.data_ptr(), dst.data_ptr(), g, S, 0.2, 0.2, "f32", outer, s, True,
                                              lead_frac=float(lf), part=part)
                return d

            info = chunk("both")
            ms = {k: [] for k in ("pass", "inner", "outer", "both")}
            for r in range(args.rounds + 1):
                n_warm = int(50e3 / max(tb(), 1.0))  # ~50 ms of passes: the clock warm-up
                for _ in range(n_warm):
                    tb()
                for k in ms:
                    us = tb() if k == "pass" else chunk(k)["kernel_us"]
                    if r > 0:
                        ms[k].append(us)
            rat = {k: round(statistics.median(a / b for a, b in zip(ms[k], ms["pass"])), 4) for k in ("inner", "outer", "both")}
            print(json.dumps({"tile": tile, "lead_frac": float(lf), "outer_wgs": info["outer_blocks"],
                              "inner_wgs": info["inner_blocks"], "band": info["band"],
                              "model": {"inner/serial": round(info["inner_cost"] / info["serial_cost"], 4),
                                        "outer/serial": round(info["outer_cost"] / info["serial_cost"], 4)},
                              "median_us": {k: round(statistics.median(v), 1) for k, v in ms.items()},
                              "over_pass": rat}), flush=True)
        del src, dst
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
