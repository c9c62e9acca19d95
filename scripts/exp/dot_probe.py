"""Dot-product grid sweep (csrc/kernels/dot.hip): 2^30 fp64 x . y, single-pass
reduction, at several workgroup counts, interleaved, plus torch.dot (the
library kernel) for comparison. Prints one JSON line per (grid, round) and a
median summary. One GPU; usage: python scripts/exp/dot_probe.py [LOG2N] [ROUNDS] [rand|ones]"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cuda_mpi_scratch_amd import hip  # noqa: E402


def main():
    log2n = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    init = sys.argv[3] if len(sys.argv) > 3 else "rand"  # rand | ones (bench.py's DotProduct data)
    n = 1 << log2n
    H = hip()
    make = torch.ones if init == "ones" else torch.rand
    x = make(n, dtype=torch.float64, device="cuda")
    y = make(n, dtype=torch.float64, device="cuda")
    out = torch.zeros(1, dtype=torch.float64, device="cuda")
    partials = torch.zeros(8192, dtype=torch.float64, device="cuda")
    counter = torch.zeros(1, dtype=torch.int32, device="cuda")
    want = torch.dot(x, y).item()
    s = torch.cuda.current_stream().cuda_stream
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    grids = [cus, 2 * cus, 3 * cus, 4 * cus, 8 * cus]
    reps = 20
    res = {g: [] for g in grids}
    res["torch"] = []
    # clock warm-up
    for _ in range(30):
        H.dot(x.data_ptr(), y.data_ptr(), n, out.data_ptr(), partials.data_ptr(), counter.data_ptr(),
              "single-pass", "f64", "f64", cus, s)
    torch.cuda.synchronize()
    for r in range(rounds):
        for g in grids + ["torch"]:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                if g == "torch":
                    torch.dot(x, y, out=out[0])
                else:
                    H.dot(x.data_ptr(), y.data_ptr(), n, out.data_ptr(), partials.data_ptr(), counter.data_ptr(),
                          "single-pass", "f64", "f64", g, s)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / reps
            rel = abs(out.item() - want) / abs(want)
            tbs = 2 * n * 8 / (us * 1e-6) / 1e12
            res[g].append(tbs)
            print(json.dumps({"grid": g, "round": r, "us": round(us, 2), "tb_s": round(tbs, 3),
                              "rel_err": rel}), flush=True)
    print(json.dumps({"summary": {str(g): round(statistics.median(v), 3) for g, v in res.items()},
                      "n": n, "cus": cus, "init": init}), flush=True)


if __name__ == "__main__":
    main()
