"""How long the after-free read slowdown lasts (dot_free_state.py) as a function
of the freed size: free G GiB, then time back-to-back 4 GiB dots (x, y of 2^28
fp64) for a few seconds and report, per 100 ms bucket, the median read rate.
One GPU; usage: python scripts/exp/free_decay.py [GIB ...]"""
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cuda_mpi_scratch_amd import hip  # noqa: E402


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [8, 32]
    H = hip()
    n = 1 << 28
    x = torch.rand(n, dtype=torch.float64, device="cuda")
    y = torch.rand(n, dtype=torch.float64, device="cuda")
    out = torch.zeros(1, dtype=torch.float64, device="cuda")
    part = torch.zeros(4096, dtype=torch.float64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream

    def dot_rate(reps=4):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            H.dot(x.data_ptr(), y.data_ptr(), n, out.data_ptr(), part.data_ptr(), cnt.data_ptr(), "single-pass",
                  "f64", "f64", 0, s)
        e1.record()
        e1.synchronize()
        return reps * 2 * n * 8 / (e0.elapsed_time(e1) * 1e-3) / 1e12

    for _ in range(200):
        dot_rate()
    base = statistics.median(dot_rate() for _ in range(50))
    print(json.dumps({"baseline_tb_s": round(base, 3)}), flush=True)
    for gib in sizes:
        d = torch.empty(gib << 28, dtype=torch.float32, device="cuda")
        d.fill_(1.0)
        torch.cuda.synchronize()
        del d
        t0 = time.perf_counter()
        torch.cuda.empty_cache()
        t_free = time.perf_counter() - t0
        buckets = {}
        while time.perf_counter() - t0 < 6.0:
            r = dot_rate()
            buckets.setdefault(int((time.perf_counter() - t0) * 10), []).append(r)
        series = [(k / 10, round(statistics.median(v), 3)) for k, v in sorted(buckets.items())]
        back = next((t for t, r in series if r > 0.99 * base), None)
        print(json.dumps({"freed_gib": gib, "free_call_s": round(t_free, 4), "recovered_at_s": back,
                          "series": series}), flush=True)
        time.sleep(1.0)


if __name__ == "__main__":
    main()
